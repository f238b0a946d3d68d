/*
 * rt_oracle.c -- CPU restatement of the reference's serial fp64 render path.
 *
 * TEST INFRASTRUCTURE ONLY (parity checker + CPU baseline).  Never linked into
 * the product library.  See rt_oracle.h for the pinning story.
 *
 * Numerics: every expression keeps the reference's operation order, operand
 * order and IEEE-754 double rounding.  Build with -ffp-contract=off (the
 * reference's own `g++ -O3` on x86-64 emits no FMA without -march).
 */
#include "rt_oracle.h"

#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#ifndef M_PI
#define M_PI 3.14159265358979323846
#endif

/* include/ray_math_constants.h:22-23 and include/scene.h:38 */
static const double ORC_EPSILON = 0.001;
static const double ORC_INFINITY = 1e20;
static const double ORC_K_SPECULAR = 0.5;

/* ---------------------------------------------------------------- vec3.h */
static inline orc_vec3 v3(double x, double y, double z) { orc_vec3 r = {x, y, z}; return r; }
static inline orc_vec3 vadd(orc_vec3 a, orc_vec3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); } /* vec3.h:13 */
static inline orc_vec3 vsub(orc_vec3 a, orc_vec3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); } /* vec3.h:14 */
static inline orc_vec3 vmul(orc_vec3 a, orc_vec3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); } /* vec3.h:15 */
static inline orc_vec3 vscale(orc_vec3 a, double t) { return v3(a.x * t, a.y * t, a.z * t); }      /* vec3.h:16 */
static inline double vlength(orc_vec3 a) { return sqrt(a.x * a.x + a.y * a.y + a.z * a.z); }      /* vec3.h:19 */
static inline orc_vec3 vnorm(orc_vec3 a) {                                                       /* vec3.h:20 */
    double len = vlength(a);
    return v3(a.x / len, a.y / len, a.z / len);
}
static inline double vdot(orc_vec3 a, orc_vec3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }  /* vec3.h:23-25 */
static inline orc_vec3 vcross(orc_vec3 a, orc_vec3 b) {                                          /* vec3.h:27-29 */
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
static inline orc_vec3 vreflect(orc_vec3 v, orc_vec3 n) {                                        /* vec3.h:31-33 */
    return vsub(v, vscale(vscale(n, 2.0), vdot(v, n)));
}
/* std::max(0.0, x) / std::min(1.0, x) as libstdc++ defines them (a<b ? b : a). */
static inline double max0(double x) { return (0.0 < x) ? x : 0.0; }
static inline double min1(double x) { return (x < 1.0) ? x : 1.0; }

/* ----------------------------------------------------------------- ray.h */
typedef struct { orc_vec3 o, d; } orc_ray;
static inline orc_ray make_ray(orc_vec3 o, orc_vec3 d) { orc_ray r; r.o = o; r.d = vnorm(d); return r; } /* ray.h:12 */

/* -------------------------------------------------------------- sphere.h */
int orc_intersect(const orc_sphere *s, orc_vec3 ro, orc_vec3 rd, double *t) {
    /* sphere.h:29-32 */
    orc_vec3 oc = vsub(ro, s->center);
    double a = vdot(rd, rd);
    double b = 2.0 * vdot(oc, rd);
    double c = vdot(oc, oc) - s->radius * s->radius;
    double disc = b * b - 4 * a * c; /* sphere.h:34: (4*a)*c */
    if (disc < 0) return 0;          /* sphere.h:37-40 */
    if (disc == 0) {                 /* sphere.h:43-47: tangent root, even if negative */
        *t = -b / (2 * a);
        return 1;
    }
    double t1 = (-b - sqrt(disc)) / (2 * a); /* sphere.h:49-50 */
    double t2 = (-b + sqrt(disc)) / (2 * a);
    double tmax = (t1 < t2) ? t2 : t1;       /* std::max(t1,t2) */
    if (tmax < 0) return 0;                  /* sphere.h:51-53 */
    double tt = (t2 < t1) ? t2 : t1;         /* std::min(t1,t2) sphere.h:54 */
    if (tt < 0) tt = tmax;                   /* sphere.h:55-57 */
    *t = tt;
    return 1;
}

/* --------------------------------------------------------------- scene.h */
/* scene.h:41-61: closest hit over all spheres in file order, strict '<'. */
static int find_intersection(const orc_scene *s, const orc_ray *r, double *t_out, int *idx_out) {
    double t = ORC_INFINITY;
    int idx = -1;
    for (int i = 0; i < s->num_spheres; i++) {
        double tt = 0;
        if (orc_intersect(&s->spheres[i], r->o, r->d, &tt)) {
            if (tt < t) { idx = i; t = tt; }
        }
    }
    *t_out = t;
    *idx_out = idx;
    return idx >= 0;
}

/* scene.h:65-86 */
static int in_shadow(const orc_scene *s, orc_vec3 p, const orc_light *L) {
    orc_vec3 to_light = vsub(L->position, p);
    double dist = vlength(to_light);
    orc_vec3 ldir = vnorm(to_light);
    orc_ray sr = make_ray(vadd(p, vscale(ldir, ORC_EPSILON)), ldir);
    double t;
    int idx;
    if (find_intersection(s, &sr, &t, &idx)) return t < dist;
    return 0;
}

/* scene.h:89-121 */
static orc_vec3 shade(const orc_scene *s, orc_vec3 p, orc_vec3 n, const orc_sphere *m, orc_vec3 view,
                      orc_counts *cnt) {
    orc_vec3 color = vmul(s->ambient, m->color);
    for (int l = 0; l < s->num_lights; l++) {
        const orc_light *L = &s->lights[l];
        cnt->shadow++;
        if (in_shadow(s, p, L)) continue;
        orc_vec3 ldir = vnorm(vsub(L->position, p));
        double ndl = max0(vdot(n, ldir));
        orc_vec3 diffuse = vscale(vscale(m->color, 1.0 - m->reflectivity), ndl);
        orc_vec3 rdir = vreflect(vscale(ldir, -1), n);
        double rdv = max0(vdot(rdir, view));
        double spec = pow(rdv, m->shininess);
        orc_vec3 specular = vscale(vscale(L->color, ORC_K_SPECULAR), spec);
        color = vadd(vadd(specular, diffuse), color); /* scene.h:117 */
    }
    return color;
}

/* ------------------------------------------------------------- main.cpp */
/* main.cpp:16-58 */
static orc_vec3 trace_ray(const orc_scene *s, const orc_ray *r, int depth, orc_counts *cnt) {
    if (depth <= 0) return v3(0, 0, 0);
    double t;
    int idx;
    if (!find_intersection(s, r, &t, &idx)) {
        double tt = 0.5 * (r->d.y + 1.0); /* main.cpp:28-29 */
        return vadd(vscale(v3(1, 1, 1), 1.0 - tt), vscale(v3(0.5, 0.7, 1.0), tt));
    }
    const orc_sphere *sp = &s->spheres[idx];
    orc_vec3 hit = vadd(r->o, vscale(r->d, t));
    orc_vec3 norm = vnorm(vsub(hit, sp->center));       /* sphere.h:62-64 */
    orc_vec3 view = vnorm(vsub(r->o, hit));             /* main.cpp:38 */
    orc_vec3 col = shade(s, hit, norm, sp, view, cnt);
    if (sp->reflectivity > 0) {                         /* main.cpp:43-55 */
        orc_vec3 rd = vsub(r->d, vscale(vscale(norm, 2.0), vdot(r->d, norm)));
        orc_ray rr = make_ray(vadd(hit, vscale(norm, ORC_EPSILON)), rd);
        if (depth - 1 >= 1) cnt->reflect++;
        orc_vec3 rc = trace_ray(s, &rr, depth - 1, cnt);
        double refl = sp->reflectivity;
        col = vadd(vscale(col, 1.0 - refl), vscale(rc, refl));
    }
    return col;
}

void orc_make_camera(const orc_scene *s, orc_camera *cam) {
    /* camera.h:10-15 */
    cam->position = s->cam_position;
    cam->forward = vnorm(vsub(s->cam_look_at, s->cam_position));
    cam->right = vnorm(vcross(cam->forward, v3(0, 1, 0)));
    cam->up = vnorm(vcross(cam->right, cam->forward));
    cam->scale = tan(s->cam_fov * 0.5 * M_PI / 180.0); /* camera.h:19 */
}

/* camera.h:17-25 */
static orc_ray get_ray(const orc_camera *c, double u, double v) {
    double aspect = 1.0;
    orc_vec3 dir = vadd(vadd(c->forward, vscale(c->right, (u - 0.5) * c->scale * aspect)),
                        vscale(c->up, (v - 0.5) * c->scale));
    return make_ray(c->position, vnorm(dir)); /* normalized, then normalized again by Ray() */
}

/* estimate_tile_complexity, src/main_hybrid.cpp:323-347: five camera rays at
 * the tile's corners and centre, u = x / img_w and v = y / img_h (the
 * reference divides by float(IMG_WIDTH) / float(IMG_HEIGHT), not W - 1), the
 * centre weighted 2, summed over every sphere whose intersect() reports a hit
 * (sphere.h:26-59; t itself is unused).  Tile = [x0, x1) x [y0, y1). */
int orc_tile_complexity(const orc_scene *s, int x0, int y0, int x1, int y1, int img_w, int img_h) {
    orc_camera cam;
    orc_make_camera(s, &cam);
    const int sx[5] = {x0, x1 - 1, (x0 + x1) / 2, x0, x1 - 1};
    const int sy[5] = {y0, y0, (y0 + y1) / 2, y1 - 1, y1 - 1};
    const int w[5] = {1, 1, 2, 1, 1};
    int cplx = 0;
    for (int i = 0; i < 5; i++) {
        orc_ray r = get_ray(&cam, (double)sx[i] / (float)img_w, (double)sy[i] / (float)img_h);
        for (int k = 0; k < s->num_spheres; k++) {
            double t;
            if (orc_intersect(&s->spheres[k], r.o, r.d, &t)) cplx += w[i];
        }
    }
    return cplx;
}

int orc_quantize(double c) {
    double m = 255.99 * min1(c); /* main.cpp:85 */
    if (m <= -2147483648.0) return -2147483647 - 1;
    return (int)m;
}

/* The pixel loop (main.cpp:146-157) over the rows of one shard; `camp` is an
 * explicit camera basis (a moved view, as a caller builds with Camera
 * directly), NULL for the scene's (main.cpp:132). */
int orc_render_cam(const orc_scene *s, const orc_camera *camp, int W, int H, int depth, int band, int first,
                   int stride, int row_count, uint8_t *rgb, double *fb, orc_counts *counts, int nthreads) {
    if (W <= 0 || H <= 0 || band <= 0 || stride <= 0 || first < 0 || row_count < 0) return -1;
    orc_camera cam;
    if (camp)
        cam = *camp;
    else
        orc_make_camera(s, &cam);
    orc_counts total = {0, 0, 0, 0};
    long long npx = (long long)row_count * W;
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        orc_counts local = {0, 0, 0, 0};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (long long p = 0; p < npx; p++) {
            int k = (int)(p / W), i = (int)(p % W);
            long long y = (long long)(k / band) * band * stride + (long long)first * band + (k % band);
            if (y >= H) continue;
            int j = H - 1 - (int)y; /* main.cpp:74: PPM row y holds reference row j */
            double u = (double)i / (W - 1); /* main.cpp:151-152 */
            double v = (double)j / (H - 1);
            orc_ray r = get_ray(&cam, u, v);
            if (depth >= 1) local.primary++;
            orc_vec3 c = trace_ray(s, &r, depth, &local);
            double ch[3] = {c.x, c.y, c.z};
            for (int q = 0; q < 3; q++) {
                if (fb) fb[p * 3 + q] = ch[q];
                int qv = orc_quantize(ch[q]);
                if (qv < 0) { local.negative++; qv = 0; }
                if (rgb) rgb[p * 3 + q] = (uint8_t)qv;
            }
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            total.primary += local.primary;
            total.shadow += local.shadow;
            total.reflect += local.reflect;
            total.negative += local.negative;
        }
    }
    if (counts) *counts = total;
    return 0;
}

int orc_render(const orc_scene *s, int W, int H, int depth, int band, int first, int stride, int row_count,
               uint8_t *rgb, double *fb, orc_counts *counts, int nthreads) {
    return orc_render_cam(s, NULL, W, H, depth, band, first, stride, row_count, rgb, fb, counts, nthreads);
}

/* The reference GPU's antialias mode (src/main_gpu.cu:249-333) restated in the
 * serial fp64 semantics: sample s = 0..samples-1 offsets (x, j) by
 * ((s % 2) * 0.5, s >= 2 ? 0.5 : 0) (main_gpu.cu:253-256), each sample is a
 * full trace_ray, the colours are summed in sample order from 0
 * (main_gpu.cu:249-327) and scaled by 1/samples (:331).  Full frame, PPM
 * row order. */
int orc_render_aa(const orc_scene *s, int W, int H, int depth, int samples, uint8_t *rgb, double *fb,
                  orc_counts *counts, int nthreads) {
    if (W <= 0 || H <= 0 || (samples != 1 && samples != 4)) return -1;
    orc_camera cam;
    orc_make_camera(s, &cam);
    orc_counts total = {0, 0, 0, 0};
    long long npx = (long long)H * W;
    if (nthreads < 1) nthreads = 1;
#ifdef _OPENMP
#pragma omp parallel num_threads(nthreads)
#endif
    {
        orc_counts local = {0, 0, 0, 0};
#ifdef _OPENMP
#pragma omp for schedule(dynamic, 64)
#endif
        for (long long p = 0; p < npx; p++) {
            int y = (int)(p / W), i = (int)(p % W);
            int j = H - 1 - y;
            orc_vec3 acc = {0.0, 0.0, 0.0};
            for (int smp = 0; smp < samples; smp++) {
                double ox = (double)(smp % 2) * 0.5, oy = smp >= 2 ? 0.5 : 0.0;
                double u = ((double)i + ox) / (W - 1);
                double v = ((double)j + oy) / (H - 1);
                orc_ray r = get_ray(&cam, u, v);
                if (depth >= 1) local.primary++;
                orc_vec3 c = trace_ray(s, &r, depth, &local);
                acc.x = acc.x + c.x;
                acc.y = acc.y + c.y;
                acc.z = acc.z + c.z;
            }
            double inv = 1.0 / (double)samples;
            double ch[3] = {acc.x * inv, acc.y * inv, acc.z * inv};
            for (int q = 0; q < 3; q++) {
                if (fb) fb[p * 3 + q] = ch[q];
                int qv = orc_quantize(ch[q]);
                if (qv < 0) { local.negative++; qv = 0; }
                if (rgb) rgb[p * 3 + q] = (uint8_t)qv;
            }
        }
#ifdef _OPENMP
#pragma omp critical
#endif
        {
            total.primary += local.primary;
            total.shadow += local.shadow;
            total.reflect += local.reflect;
            total.negative += local.negative;
        }
    }
    if (counts) *counts = total;
    return 0;
}

/* ------------------------------------------------------- scene_loader.h */
/* Emulates `std::istream >> double` (libstdc++ num_get): greedy accumulation of
 * [sign] digits [. digits] [e [sign] digits], then strtod over exactly that
 * text; incomplete text, or +-inf from overflow, is a failure. */
static int read_double(const char **pp, const char *end, double *out) {
    const char *p = *pp;
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\v' || *p == '\f')) p++;
    char buf[512];
    size_t n = 0;
    const char *q = p;
    if (q < end && (*q == '+' || *q == '-')) buf[n++] = *q++;
    int seen_dot = 0, seen_e = 0;
    while (q < end && n < sizeof(buf) - 2) {
        char ch = *q;
        if (ch >= '0' && ch <= '9') { buf[n++] = ch; q++; }
        else if (ch == '.' && !seen_dot && !seen_e) { seen_dot = 1; buf[n++] = ch; q++; }
        else if ((ch == 'e' || ch == 'E') && !seen_e) {
            seen_e = 1; buf[n++] = ch; q++;
            if (q < end && (*q == '+' || *q == '-')) buf[n++] = *q++;
        } else break;
    }
    buf[n] = 0;
    *pp = q;
    if (n == 0) return 0;
    char *sanity;
    errno = 0;
    double v = strtod(buf, &sanity);
    if (sanity == buf || *sanity != 0) return 0;
    if (isinf(v)) return 0;
    *out = v;
    return 1;
}

static int read_word(const char **pp, const char *end, char *w, size_t cap) {
    const char *p = *pp;
    while (p < end && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\v' || *p == '\f')) p++;
    size_t n = 0;
    while (p < end && !(*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r' || *p == '\v' || *p == '\f')) {
        if (n + 1 < cap) w[n++] = *p;
        p++;
    }
    w[n] = 0;
    *pp = p;
    return n > 0;
}

static int read_doubles(const char **pp, const char *end, double *v, int k) {
    for (int i = 0; i < k; i++)
        if (!read_double(pp, end, &v[i])) return 0;
    return 1;
}

int orc_parse_scene(const char *text, orc_scene *out, int verbose) {
    memset(out, 0, sizeof(*out));
    out->cam_look_at = v3(0, 0, -1); /* CameraConfig() scene.h:22 */
    out->cam_fov = 60.0;
    int cap_s = 16, cap_l = 4;
    out->spheres = (orc_sphere *)malloc(sizeof(orc_sphere) * cap_s);
    out->lights = (orc_light *)malloc(sizeof(orc_light) * cap_l);
    const char *p = text;
    const char *tend = text + strlen(text);
    int line_number = 0;
    while (p < tend) { /* std::getline loop, scene_loader.h:41 */
        const char *nl = memchr(p, '\n', (size_t)(tend - p));
        const char *le = nl ? nl : tend;
        const char *ls = p;
        p = nl ? nl + 1 : tend;
        line_number++;
        if (le == ls || *ls == '#') continue;                 /* :45-47 */
        while (ls < le && (*ls == ' ' || *ls == '\t')) ls++;  /* :50-54 */
        if (ls == le) continue;
        if (*ls == '#') continue;                             /* :57-59 */
        const char *q = ls;
        char type[64];
        read_word(&q, le, type, sizeof type);
        double v[10];
        if (strcmp(type, "sphere") == 0) {                    /* :65-84 */
            if (!read_doubles(&q, le, v, 10)) {
                if (verbose) fprintf(stderr, "Warning: Invalid sphere at line %d, skipping\n", line_number);
                out->warnings++;
                continue;
            }
            if (out->num_spheres == cap_s) { cap_s *= 2; out->spheres = (orc_sphere *)realloc(out->spheres, sizeof(orc_sphere) * cap_s); }
            orc_sphere *s = &out->spheres[out->num_spheres++];
            s->center = v3(v[0], v[1], v[2]);
            s->radius = v[3];
            s->color = v3(v[4], v[5], v[6]);
            s->reflectivity = v[7]; /* metallic; v[8] roughness dropped */
            s->shininess = v[9];
        } else if (strcmp(type, "light") == 0) {              /* :85-99 */
            if (!read_doubles(&q, le, v, 7)) {
                if (verbose) fprintf(stderr, "Warning: Invalid light at line %d, skipping\n", line_number);
                out->warnings++;
                continue;
            }
            if (out->num_lights == cap_l) { cap_l *= 2; out->lights = (orc_light *)realloc(out->lights, sizeof(orc_light) * cap_l); }
            orc_light *L = &out->lights[out->num_lights++];
            L->position = v3(v[0], v[1], v[2]);
            L->color = v3(v[3], v[4], v[5]);
            L->intensity = v[6];
        } else if (strcmp(type, "ambient") == 0) {            /* :100-110 */
            if (!read_doubles(&q, le, v, 3)) {
                if (verbose) fprintf(stderr, "Warning: Invalid ambient at line %d, skipping\n", line_number);
                out->warnings++;
                continue;
            }
            out->ambient = v3(v[0], v[1], v[2]);
        } else if (strcmp(type, "camera") == 0) {             /* :111-124 */
            if (!read_doubles(&q, le, v, 7)) {
                if (verbose) fprintf(stderr, "Warning: Invalid camera at line %d, skipping\n", line_number);
                out->warnings++;
                continue;
            }
            out->cam_position = v3(v[0], v[1], v[2]);
            out->cam_look_at = v3(v[3], v[4], v[5]);
            out->cam_fov = v[6];
            out->has_camera = 1;
        } else {                                              /* :125-128 */
            if (verbose) fprintf(stderr, "Warning: Unknown type '%s' at line %d, skipping\n", type, line_number);
            out->warnings++;
        }
    }
    if (verbose) printf("Loaded scene: %d spheres, %d lights\n", out->num_spheres, out->num_lights); /* :131-132 */
    return 0;
}

int orc_load_scene(const char *path, orc_scene *out, int verbose) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        memset(out, 0, sizeof(*out));
        return -1;
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *buf = (char *)malloc((size_t)n + 1);
    size_t got = fread(buf, 1, (size_t)n, f);
    fclose(f);
    buf[got] = 0;
    /* getline stops at an embedded NUL only for the C-string view; scene files are text. */
    int rc = orc_parse_scene(buf, out, verbose);
    free(buf);
    return rc;
}

void orc_free_scene(orc_scene *s) {
    free(s->spheres);
    free(s->lights);
    s->spheres = NULL;
    s->lights = NULL;
    s->num_spheres = s->num_lights = 0;
}

/* main.cpp:69-91: "P3\n<W> <H>\n255\n" then "r g b\n" per pixel, top row first. */
int orc_write_p3(const char *path, const uint8_t *rgb, int W, int H) {
    FILE *f = fopen(path, "wb");
    if (!f) return -1;
    fprintf(f, "P3\n%d %d\n255\n", W, H);
    long long n = (long long)W * H;
    for (long long i = 0; i < n; i++) fprintf(f, "%d %d %d\n", rgb[3 * i], rgb[3 * i + 1], rgb[3 * i + 2]);
    fclose(f);
    return 0;
}
