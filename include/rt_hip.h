/*
 * rt_hip.h -- C-ABI of the MI355X (gfx950) render-loop library, librt_hip.so.
 *
 * Drop-in boundary for the per-pixel render loop of shininglegend/cs420-ray-tracer.
 * Plain C, POD structs, plain pointers and sizes; no HIP/torch types appear in
 * any signature (streams are passed as `void *` = hipStream_t).
 *
 * What each entry point replaces in the reference (file:line):
 *   rt_scene_load / rt_scene_parse  <- load_scene()           include/scene_loader.h:27-135
 *   rt_scene_free                   <- Scene destructor       include/scene.h:28-33
 *   rt_camera_from_scene            <- Camera::Camera()       include/camera.h:10-15 (+ scale of get_ray, :18-19)
 *   rt_create / rt_destroy          <- GPUResources ctor/dtor src/main_hybrid.cpp:182-195, 300-316
 *   rt_upload_scene                 <- GPUResources::upload_scene + upload_lights_and_ambience
 *                                      src/main_hybrid.cpp:198-279, src/kernel.cu:202-207
 *   rt_render                       <- the serial pixel loop  src/main.cpp:146-157 (trace_ray :16-58),
 *                                      the OpenMP loop :185-199, and launch_gpu_kernel src/kernel.cu:185-200
 *   rt_render_async                 <- launch_gpu_kernel(..., cudaStream_t) src/kernel.cu:185-200
 *   rt_render_frames_async          <- (new) the pixel loop over a sequence of frames in one launch
 *                                      (frame f = rt_render_async with cams[f])
 *   rt_write_ppm                    <- write_ppm()            src/main.cpp:69-91
 *   rt_kernel_times                 <- cudaEventElapsedTime around the kernel, src/main_gpu.cu:496-519
 *   rt_unpermute_rows               <- (new) reassembly of the multi-GPU row shards
 *   rt_render_tiles                 <- the same for a list of tiles in one launch (the hybrid driver's GPU share)
 *   rt_render_tile                  <- launch_gpu_kernel's tile semantics  src/kernel.cu:185-200 (x = tile_x + ...,
 *                                      y = tile_y + ..., fb[y*W + x], kernel.cu:99-112), as main_hybrid.cpp:457-470
 *                                      calls it; float3 / Vec3 / RGB8 framebuffers
 *   rt_set_antialias                <- the `-a` flag of ray_gpu, src/main_gpu.cu:249-333, 363-370
 *   rt_get_info                     <- (new) the host-side builds the render calls made (camera grid,
 *                                      tile launch order) and their cost
 *   launch_gpu_kernel, upload_lights_and_ambience (include/rt_hip_compat.h)
 *                                   <- the same symbols of src/kernel.cu:185-207, link-compatible
 *
 * Errors: every call returns an rt_status (0 = ok); the library never exits
 * (the reference's CUDA_CHECK -> exit(1), src/main_gpu.cu:27-35, is not kept).
 * Threading: one rt_ctx per device per host thread; distinct contexts are
 * independent and may be used concurrently.
 * Streams: all device work of a context (renders, rt_unpermute_rows) is
 * enqueued on ONE stream, the context's current stream, and is ordered only
 * on it.  The context's own stream (the default) is a BLOCKING stream: it is
 * ordered with the legacy NULL stream, so device buffers a caller fills or
 * reads on the NULL stream are ordered with the context's work.  A caller
 * that uses another stream of its own either passes it to rt_set_stream or
 * orders it against the context's stream itself.
 */
#ifndef RT_HIP_H
#define RT_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RT_HIP_ABI_VERSION 12 /* 4: the reference hybrid interface (rt_hip_compat.h); 5: rt_rows_for_shard;
                                   6: rt_render_tiles; 7: rt_get_info; 8: rt_info sphere-grid fields;
                                   9: rt_info behind-grid fields; 10: RT_ERR_CHECK;
                                   11: rt_info BVH / light-grid build times, scratch bytes;
                                   12: rt_info shadow_line_bounded */
/* Longest reflection chain the GPU path keeps per pixel (depth <= RT_MAX_DEPTH). */
#define RT_MAX_DEPTH 64

typedef enum rt_status {
    RT_OK = 0,
    RT_ERR_INVALID_ARG = 1,
    RT_ERR_NO_DEVICE = 2,
    RT_ERR_HIP = 3,          /* a HIP runtime call failed; see rt_last_error() */
    RT_ERR_OUT_OF_MEMORY = 4,
    RT_ERR_NO_SCENE = 5,     /* rt_render before rt_upload_scene */
    RT_ERR_IO = 6,           /* scene file could not be opened / image not written */
    RT_ERR_DEPTH = 7,        /* depth > RT_MAX_DEPTH */
    RT_ERR_CHECK = 8,        /* bounds-checked build (-DRT_CHECK) only: a device index into a host-built
                                structure was out of range; rt_last_error() names the site (rt_render_stats) */
} rt_status;

/* Sphere + Material, include/sphere.h:8-21.  reflectivity = the file's
 * "metallic" column (scene_loader.h:288); roughness is dropped as upstream. */
typedef struct rt_sphere {
    double center[3];
    double radius;
    double color[3];
    double reflectivity;
    double shininess;
} rt_sphere;

/* Light, include/scene.h:10-14 (intensity is parsed but unused, scene.h:117). */
typedef struct rt_light {
    double position[3];
    double color[3];
    double intensity;
} rt_light;

/* Scene + CameraConfig, include/scene.h:17-38. */
typedef struct rt_scene {
    int32_t num_spheres;
    int32_t num_lights;
    rt_sphere *spheres;
    rt_light *lights;
    double ambient[3];        /* default (0,0,0) */
    double cam_position[3];   /* default (0,0,0)   scene.h:22 */
    double cam_look_at[3];    /* default (0,0,-1)  scene.h:22 */
    double cam_fov;           /* default 60        scene.h:22 */
    int32_t has_camera;
    int32_t warnings;         /* records skipped by the parser */
} rt_scene;

/* Camera basis computed on the host (camera.h:10-15); scale = tan(fov*0.5*M_PI/180). */
typedef struct rt_camera {
    double position[3];
    double forward[3];
    double right[3];
    double up[3];
    double scale;
} rt_camera;

/* Which image rows a call renders.  Output row k (0 <= k < count) is image row
 *   y = (k / band) * band * stride + first * band + (k % band)
 * in PPM order (y = 0 is the TOP row, i.e. reference row j = H-1-y,
 * src/main.cpp:74).  Rows with y >= H are padding: they are written as zeros.
 * Full frame: {band=1, first=0, stride=1, count=H}.  Rank r of G GPUs with
 * cyclic bands of B rows: {B, r, G, ceil(ceil(H/B)/G)*B}. */
typedef struct rt_rows {
    int32_t band;
    int32_t first;
    int32_t stride;
    int32_t count;
} rt_rows;

/* The multi-GPU row layout every driver uses -- ray_hip --gpus G,
 * bench.py's torch.distributed ranks, rt_unpermute_rows: rank `rank` of
 * `num_shards` renders the cyclic bands of `band` rows rank, rank + G, ...;
 * every rank gets the same row count ceil(ceil(H / band) / G) * band (rows past
 * the image are padding).  Fails for band < 1, G < 1, rank outside [0, G). */
int rt_rows_for_shard(int height, int band, int rank, int num_shards, rt_rows *out);

/* Ray counts: primary = pixels traced; shadow = lights x shaded
 * hits (counted even when the GPU exits early); reflect = reflection rays
 * traced (reflective hit with depth-1 >= 1).  kernel_ms = HIP-event time of the
 * render kernel(s) on the context's stream. */
typedef struct rt_stats {
    uint64_t rays_primary;
    uint64_t rays_shadow;
    uint64_t rays_reflect;
    uint64_t negative_clamped; /* channels whose int(255.99*min(1,c)) < 0, stored as 0 */
    double kernel_ms;
    uint64_t tests_exact;      /* exact ray-sphere tests executed (sphere.h:26-59), live lanes only */
    uint64_t tests_cull;       /* sphere-vs-wave-bound tests (one per sphere per wave sweep) */
} rt_stats;

typedef struct rt_ctx rt_ctx;

/* ---- host-side scene / camera / image I/O (no GPU needed) ---------------- */
int rt_scene_load(const char *path, rt_scene *out, int verbose);
int rt_scene_parse(const char *text, rt_scene *out, int verbose);
void rt_scene_free(rt_scene *scene);
int rt_camera_from_scene(const rt_scene *scene, rt_camera *out);
/* binary=0: P3 text byte-identical to write_ppm (src/main.cpp:69-91); binary=1: P6. */
int rt_write_ppm(const char *path, const uint8_t *rgb, int width, int height, int binary);
const char *rt_error_string(int status);
int rt_abi_version(void);

/* ---- device ------------------------------------------------------------- */
int rt_device_count(int *count);
int rt_create(int device, rt_ctx **out);
void rt_destroy(rt_ctx *ctx);
const char *rt_last_error(const rt_ctx *ctx);
/* Use an external stream (hipStream_t) for all later work of this context;
 * NULL restores the context's own (blocking) stream.  The switch is ordered:
 * work enqueued after it on the new stream waits for all work already
 * enqueued on the previous stream (the context's scratch buffers are shared
 * by every launch). */
int rt_set_stream(rt_ctx *ctx, void *hip_stream);
/* Per-wave conservative sphere culling (default on).  Off = every ray tests
 * every sphere (the reference's brute-force sweep, scene.h:47-58).  Output
 * bytes are identical either way; only the work differs. */
int rt_set_culling(rt_ctx *ctx, int enable);
/* Copies the scene into device memory owned by the context (replaces any
 * previous scene).  The host arrays may be freed afterwards. */
int rt_upload_scene(rt_ctx *ctx, const rt_scene *scene);

/* Synchronous render.  rgb_out: rows->count * width * 3 bytes, PPM row order
 * (see rt_rows).  out_on_device = 1 if rgb_out is device memory of this
 * context's device, 0 for host memory.  rows = NULL means the full frame.
 * stats may be NULL. */
int rt_render(rt_ctx *ctx, const rt_camera *cam, int width, int height, int depth, const rt_rows *rows,
              uint8_t *rgb_out, int out_on_device, rt_stats *stats);
/* Asynchronous render into DEVICE memory on the context's stream.  The kernels
 * are only enqueued, but host-side work can happen inside the call and then
 * wait for the context's stream first (work in flight may still read the
 * buffer being replaced):
 *   - the tile launch order (rt_sched), rebuilt when the view, the image or
 *     shard geometry or the scene changed since the previous launch (~0.1 ms);
 *   - the camera grid's cube-map tables and buffers, the first time a grid
 *     size is used.  The camera grids themselves (closest hits of camera rays)
 *     are built on the device ahead of the render kernel, per camera position,
 *     for a multi-frame launch (one grid per distinct position) or a one-frame
 *     launch at the previous launch's position (~0.05 ms, cached).
 * rt_get_info() reports both.  rt_render_stats() waits for the stream and
 * returns the stats of the most recent rt_render_async. */
int rt_render_async(rt_ctx *ctx, const rt_camera *cam, int width, int height, int depth, const rt_rows *rows,
                    uint8_t *rgb_out_device);
int rt_render_stats(rt_ctx *ctx, rt_stats *stats);

/* Most frames one rt_render_frames_async launch renders. */
#define RT_MAX_FRAMES 32
/* Asynchronous render of `nframes` frames (1..RT_MAX_FRAMES) of the uploaded
 * scene in ONE kernel launch, frame f seen through cams[f]: a frame sequence
 * of the per-frame pixel loop src/main.cpp:146-157, each frame exactly what
 * rt_render_async(ctx, &cams[f], ...) writes, into DEVICE memory at
 * rgb_out_device + f * frame_stride (frame_stride >= rows' count * width * 3
 * bytes).  The tiles of all frames share one launch, so the long reflection
 * chains of one frame overlap the others' work instead of each frame ending
 * on its slowest tiles.  Counts as ONE launch for rt_kernel_times; the stats
 * of rt_render_stats are the sums over its frames.  The context's scratch
 * (reflection stack, deferred-ray queue) grows to the largest launch seen, so
 * launches of as many frames or fewer do not re-allocate: render the largest
 * batch once before timing a sequence. */
int rt_render_frames_async(rt_ctx *ctx, const rt_camera *cams, int nframes, int width, int height, int depth,
                           const rt_rows *rows, uint8_t *rgb_out_device, size_t frame_stride);

/* Durations (ms, HIP events recorded in-stream around each render kernel) of
 * the render launches issued since the previous call, oldest first, at most
 * max_n (and at most the 256 most recent).  Waits for the context stream. */
int rt_kernel_times(rt_ctx *ctx, double *ms_out, int max_n, int *n_out);

/* Framebuffer formats of rt_render_tile. */
#define RT_FB_RGB8 0  /* uint8 RGB, width*height*3, PPM row order (top row first), quantised as write_ppm */
#define RT_FB_F32X3 1 /* float RGB per pixel at index y*width + x, y = 0 the BOTTOM row: the reference's
                         d_framebuffer of launch_gpu_kernel (kernel.cu:112), unquantised */
#define RT_FB_F64X3 2 /* double RGB (Vec3) per pixel, same indexing: the serial framebuffer, main.cpp:156 */

/* launch_gpu_kernel (src/kernel.cu:185-200) with its tile semantics: renders
 * pixels x in [tile_x, tile_x + tile_w), y in [tile_y, tile_y + tile_h)
 * (clipped to the image; y counts from the bottom row, v = y/(H-1)) into a
 * full-image DEVICE framebuffer of the given format; other pixels are not
 * touched.  Asynchronous on the context stream, like the reference; the
 * caller synchronises (rt_render_stats waits and returns this tile's counts).
 * The colours are the serial path's (fp64, A1-A13), not the reference CUDA
 * kernel's fp32 approximation. */
int rt_render_tile(rt_ctx *ctx, const rt_camera *cam, int image_width, int image_height, int depth, int tile_x,
                   int tile_y, int tile_width, int tile_height, int fb_format, void *fb_device);

/* One launch_gpu_kernel tile (kernel.cu:185-200): pixels x in [x, x + width),
 * framebuffer rows j in [y, y + height) (j = 0 the bottom row). */
typedef struct rt_tile {
    int32_t x, y, width, height;
} rt_tile;

/* Many tiles in ONE launch (a hybrid driver's GPU share of a frame,
 * main_hybrid.cpp:457-470 / 535-548, without a launch and a sync per tile):
 * every 8x8-pixel block of the image that overlaps a tile is rendered into the
 * full-image DEVICE framebuffer exactly as rt_render_tile renders it, so the
 * tiles' pixels are rt_render_tile's; the other pixels of those blocks are
 * written too (with their own colours), all others are not touched.
 * Asynchronous on the context stream; waits for the stream first when the
 * context's block list is still in use. */
int rt_render_tiles(rt_ctx *ctx, const rt_camera *cam, int image_width, int image_height, int depth,
                    const rt_tile *tiles, int num_tiles, int fb_format, void *fb_device);

/* Samples per pixel for later renders: 1 (default, the serial path) or 4 (the
 * reference GPU's `-a` antialias mode, main_gpu.cu:249-333: offsets
 * (0,0) (0.5,0) (0,0.5) (0.5,0.5) added to (x, y) before u = x/(W-1),
 * v = y/(H-1); the 4 colours summed in that order and scaled by 1/4, all in
 * the serial fp64 semantics).  Ray counts include every sample. */
int rt_set_antialias(rt_ctx *ctx, int samples);

/* Host-side work of the render calls since rt_create (see rt_render_async). */
typedef struct rt_info {
    int32_t cam_grid_last;       /* 1: the most recent launch traced its camera rays on a camera grid */
    int32_t cam_grid_n;          /* its cells per cube-map face edge (0: none) */
    uint64_t cam_grid_builds;    /* camera grids built */
    double cam_grid_build_ms;    /* host wall time of those builds (incl. the stream wait and the upload) */
    uint64_t tile_order_builds;  /* tile launch orders built */
    double tile_order_build_ms;  /* host wall time of those builds */
    double upload_ms;            /* host wall time of the most recent rt_upload_scene (BVH, light grids, copies) */
    uint64_t launches;           /* render launches enqueued */
    int32_t sphere_grids;        /* spheres with a sphere grid (reflection rays' closest hit; 0: none) */
    int32_t sphere_grid_n;       /* their cells per cube-map face edge */
    uint64_t sphere_grid_entries;  /* list entries of all sphere grids (8 bytes each) */
    double sphere_grid_build_ms; /* host wall time of their build (by the scene's first multi-frame or second launch) */
    int32_t behind_grid;         /* 1: the scene has a behind grid (closest-hit lines' part behind their origin) */
    int32_t behind_grid_last;    /* 1: the most recent launch's BVH walks used it */
    uint64_t behind_grid_cells;  /* its cells */
    uint64_t behind_grid_entries;  /* its list entries (20 bytes each) */
    double behind_grid_build_ms; /* host wall time of its build, part of upload_ms */
    double bvh_build_ms;         /* host wall time of the BVH build and upload, part of upload_ms */
    double light_grid_build_ms;  /* host wall time of the light grids' build and upload, part of upload_ms */
    uint64_t scratch_bytes;      /* device scratch the context holds for its launches: reflection stacks (stack
                                    homes / per-pixel stack), the deferred queue, the camera grids, the tile order */
    int32_t shadow_line_bounded; /* 1: the scene's bound keeps every shadow line within its light grid's margin, so
                                    the per-ray check is skipped (rt_device.h shadow_cells off_free); 0: checked */
    int32_t reserved0;
} rt_info;
int rt_get_info(rt_ctx *ctx, rt_info *out);

/* Reassemble G shards gathered rank-major ([G][rows_per_rank][W][3], rank r
 * rendered with rt_rows{band, r, G, rows_per_rank}) into a PPM-ordered
 * [H][W][3] image.  Both pointers are device memory; runs on the ctx stream. */
int rt_unpermute_rows(rt_ctx *ctx, const uint8_t *gathered_device, uint8_t *image_device, int width, int height,
                      int band, int num_shards, int rows_per_shard);

#ifdef __cplusplus
}
#endif
#endif /* RT_HIP_H */
