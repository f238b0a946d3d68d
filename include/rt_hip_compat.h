/*
 * rt_hip_compat.h -- the reference's hybrid GPU interface, link-compatible,
 * exported by librt_hip.so.
 *
 * The reference's CPU+GPU driver (src/main_hybrid.cpp) declares and calls two
 * C functions that src/kernel.cu implements:
 *
 *   extern "C" void launch_gpu_kernel(float3 *d_framebuffer, GPUSphere *d_spheres,
 *       int num_spheres, int num_lights, GPUCamera *camera, int tile_x, int tile_y,
 *       int tile_width, int tile_height, int image_width, int image_height,
 *       int max_depth, cudaStream_t stream);              main_hybrid.cpp:104-109, kernel.cu:185-200
 *   extern "C" void upload_lights_and_ambience(GPULight *lights, int count,
 *       float3 ambience);                                  main_hybrid.cpp:170-171, kernel.cu:202-207
 *
 * librt_hip.so exports both symbols with the same C ABI: the structs below
 * have the layouts of float3, GPUMaterial, GPUSphere, GPULight and GPUCamera
 * (include/gpu_shared.h:84-171: 12, 20, 36, 28 and 88 bytes), and a stream
 * handle is a pointer.  A caller written against the reference links against
 * librt_hip.so unchanged.
 *
 * Semantics:
 *  - upload_lights_and_ambience copies `count` lights (a HOST array, as in
 *    the reference) and the ambient colour into the state of the calling
 *    thread's current HIP device (the reference's __constant__ module state).
 *  - launch_gpu_kernel renders pixels x in [tile_x, tile_x + tile_width),
 *    y in [tile_y, tile_y + tile_height), clipped to the image, y = 0 the
 *    BOTTOM row (v = y / (H - 1)), into the caller's DEVICE float3
 *    framebuffer at index y * image_width + x (kernel.cu:99-112), on
 *    `stream`, asynchronously.  Other pixels are not touched.  d_spheres
 *    (num_spheres GPUSpheres) and camera (one GPUCamera) are DEVICE pointers,
 *    as in the reference; the first num_lights uploaded lights are used.
 *  - The colours are the SERIAL path's (fp64, src/main.cpp:16-58 with
 *    scene.h / sphere.h), evaluated on the caller's fp32 scene values
 *    promoted to double -- not the reference CUDA kernel's fp32
 *    approximation -- and rounded to float on store.  The
 *    camera basis is re-derived in fp64 from GPUCamera.origin / .forward /
 *    .fov as camera.h:10-25 does from (look_at - position); GPUCamera's other
 *    fields are unused.
 *  - Both functions return void like the reference but never exit(): the
 *    status of the calling thread's last compat call is rt_compat_status()
 *    (an rt_status; RT_ERR_INVALID_ARG for a bad argument, e.g. num_lights
 *    larger than the uploaded count, in which case nothing is rendered).
 *  - The scene is re-read from d_spheres at every launch (num_spheres x 36 B,
 *    on `stream`, which is synchronised first); the acceleration structures
 *    are rebuilt only when the spheres or the lights changed.
 */
#ifndef RT_HIP_COMPAT_H
#define RT_HIP_COMPAT_H

#ifdef __cplusplus
extern "C" {
#endif

typedef struct rt_float3 { float x, y, z; } rt_float3;                            /* float3 */
typedef struct rt_gpu_material { rt_float3 albedo; float metallic; float shininess; } rt_gpu_material;
typedef struct rt_gpu_sphere { rt_float3 center; float radius; rt_gpu_material material; } rt_gpu_sphere;
typedef struct rt_gpu_light { rt_float3 position; rt_float3 color; float intensity; } rt_gpu_light;
typedef struct rt_gpu_camera {
    rt_float3 origin, lower_left, horizontal, vertical; /* lower_left .. vertical: unused (as upstream) */
    rt_float3 forward, right, up;                       /* right, up: re-derived from forward in fp64 */
    float fov;
} rt_gpu_camera;

void launch_gpu_kernel(rt_float3 *d_framebuffer, rt_gpu_sphere *d_spheres, int num_spheres, int num_lights,
                       rt_gpu_camera *camera, int tile_x, int tile_y, int tile_width, int tile_height,
                       int image_width, int image_height, int max_depth, void *stream);
void upload_lights_and_ambience(rt_gpu_light *lights, int count, rt_float3 ambience);
/* rt_status of the calling thread's last launch_gpu_kernel / upload_lights_and_ambience. */
int rt_compat_status(void);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_COMPAT_H */
