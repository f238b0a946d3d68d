/*
 * rt_oracle.h -- CPU restatement of the reference tracer's per-pixel render loop.
 *
 * TEST INFRASTRUCTURE ONLY.  This is the parity checker ("oracle") for the HIP
 * path.  Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg
 * may load it.  The product library (librt_hip.so) never links or calls it.
 *
 * Every routine restates the serial fp64 path of shininglegend/cs420-ray-tracer
 * (the `ray_serial` binary).  Citations are <file>:<line> in the reference.
 *
 * Parity is PINNED: the restatement is checked byte-for-byte against
 *  (1) the reference's own `ray_serial` compiled from its sources
 *      (oracle/Makefile -> oracle/_ref/ray_serial, native 1280x720 d10), and
 *  (2) the reference's trace_ray compiled into oracle/ref_driver.cpp
 *      (oracle/_ref/ref_render, any size), and
 *  (3) the SHA-256 values recorded in SURVEY.md section 8(c).
 */
#ifndef RT_ORACLE_H
#define RT_ORACLE_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct { double x, y, z; } orc_vec3;

/* include/sphere.h:8-12 (Material) + sphere.h:17-21 (Sphere). */
typedef struct {
    orc_vec3 center;
    double radius;
    orc_vec3 color;
    double reflectivity; /* = "metallic" column, scene_loader.h:288 */
    double shininess;
} orc_sphere;

/* include/scene.h:10-14 */
typedef struct {
    orc_vec3 position;
    orc_vec3 color;
    double intensity; /* parsed but unused by shading (scene.h:117) */
} orc_light;

/* include/scene.h:28-38 + CameraConfig scene.h:17-25 */
typedef struct {
    int num_spheres;
    orc_sphere *spheres;
    int num_lights;
    orc_light *lights;
    orc_vec3 ambient;       /* default (0,0,0): Vec3() in vec3.h:10 */
    orc_vec3 cam_position;  /* default (0,0,0)  scene.h:22 */
    orc_vec3 cam_look_at;   /* default (0,0,-1) scene.h:22 */
    double cam_fov;         /* default 60       scene.h:22 */
    int has_camera;
    int warnings;           /* malformed / unknown records skipped */
} orc_scene;

typedef struct {
    uint64_t primary;   /* rays cast by camera.get_ray (one per pixel, depth >= 1) */
    uint64_t shadow;    /* in_shadow calls: lights x shaded hits (scene.h:96-98)   */
    uint64_t reflect;   /* reflection rays actually traced (main.cpp:43-50, depth-1 >= 1) */
    uint64_t negative;  /* channels whose int(255.99*min(1,c)) was < 0 (stored as 0) */
} orc_counts;

/* Camera basis: include/camera.h:10-15 and get_ray scale, camera.h:18-19. */
typedef struct {
    orc_vec3 position, forward, right, up;
    double scale; /* tan(fov * 0.5 * M_PI / 180.0) evaluated with glibc tan */
} orc_camera;

/* scene_loader.h:27-135.  Returns 0 on success, -1 if the file cannot be opened
 * (the reference throws std::runtime_error there, scene_loader.h:33-35). */
int orc_load_scene(const char *path, orc_scene *out, int verbose);
/* Same parser over an in-memory text. */
int orc_parse_scene(const char *text, orc_scene *out, int verbose);
void orc_free_scene(orc_scene *s);

void orc_make_camera(const orc_scene *s, orc_camera *cam);

/* Sphere::intersect, include/sphere.h:26-59.  Returns 1 on hit and writes *t. */
int orc_intersect(const orc_sphere *s, orc_vec3 ro, orc_vec3 rd, double *t);

/* Full-frame / row-subset render.
 *   Output rows are in PPM order (top row first): output row k holds image row
 *   y = (k / band) * band * stride + first * band + (k % band), and reference row
 *   j = H-1-y (main.cpp:74 writes j = H-1 .. 0).  Rows with y >= H are skipped
 *   (left untouched).  `band`,`stride` >= 1.
 *   rgb: row_count*W*3 bytes (nullable); fb: row_count*W*3 doubles (nullable).
 *   nthreads > 1 uses OpenMP dynamic scheduling (main.cpp:185) if compiled in. */
int orc_render(const orc_scene *s, int W, int H, int depth,
               int band, int first, int stride, int row_count,
               uint8_t *rgb, double *fb, orc_counts *counts, int nthreads);
/* The same with an explicit camera basis (NULL: the scene's camera). */
int orc_render_cam(const orc_scene *s, const orc_camera *cam, int W, int H, int depth, int band, int first,
                   int stride, int row_count, uint8_t *rgb, double *fb, orc_counts *counts, int nthreads);

/* Antialias mode of src/main_gpu.cu:249-333 in serial fp64 semantics: samples
 * = 1 or 4, full frame in PPM row order (see rt_oracle.c). */
int orc_render_aa(const orc_scene *s, int W, int H, int depth, int samples, uint8_t *rgb, double *fb,
                  orc_counts *counts, int nthreads);

/* estimate_tile_complexity of the hybrid driver, src/main_hybrid.cpp:323-347. */
int orc_tile_complexity(const orc_scene *s, int x0, int y0, int x1, int y1, int img_w, int img_h);

/* Quantiser of main.cpp:85-87: int(255.99 * std::min(1.0, c)). */
int orc_quantize(double c);

/* P3 writer byte-identical to main.cpp:69-91, from PPM-ordered RGB8. */
int orc_write_p3(const char *path, const uint8_t *rgb, int W, int H);

#ifdef __cplusplus
}
#endif
#endif
