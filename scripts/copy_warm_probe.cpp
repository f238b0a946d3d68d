#include <hip/hip_runtime.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>
static double now(){return std::chrono::duration<double,std::milli>(std::chrono::steady_clock::now().time_since_epoch()).count();}
int main(int argc,char**argv){
  int mode=atoi(argv[1]);
  double t=now(); hipStream_t s; hipStreamCreate(&s); printf("stream %.2f\n",now()-t);
  void*d; hipMalloc(&d, 8<<20);
  std::vector<char> h(8<<20, 1);
  auto T=[&](const char*n, auto f){double t0=now(); f(); hipStreamSynchronize(s); printf("%-28s %.3f ms\n",n,now()-t0);};
  if(mode==1){ T("warm sync H2D 8B",[&]{hipMemcpy(d,h.data(),8,hipMemcpyHostToDevice);}); T("warm sync D2H 8B",[&]{hipMemcpy(h.data(),d,8,hipMemcpyDeviceToHost);}); }
  if(mode==2){ T("warm async H2D 1MB",[&]{hipMemcpyAsync(d,h.data(),1<<20,hipMemcpyHostToDevice,s);}); T("warm async D2H 1MB",[&]{hipMemcpyAsync(h.data(),d,1<<20,hipMemcpyDeviceToHost,s);}); }
  if(mode==3){ T("warm async H2D 8B",[&]{hipMemcpyAsync(d,h.data(),8,hipMemcpyHostToDevice,s);}); T("warm async D2H 8B",[&]{hipMemcpyAsync(h.data(),d,8,hipMemcpyDeviceToHost,s);}); }
  T("sync H2D 4KB",[&]{hipMemcpy(d,h.data(),4096,hipMemcpyHostToDevice);});
  T("sync H2D 4KB again",[&]{hipMemcpy(d,h.data(),4096,hipMemcpyHostToDevice);});
  T("async D2H 6MB",[&]{hipMemcpyAsync(h.data(),d,6<<20,hipMemcpyDeviceToHost,s);});
  T("async D2H 6MB again",[&]{hipMemcpyAsync(h.data(),d,6<<20,hipMemcpyDeviceToHost,s);});
  return 0;}
