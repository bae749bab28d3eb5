/*
 * srt_oracle.c -- CPU restatement of the render hot path. TEST INFRASTRUCTURE ONLY (see
 * srt_oracle.h for who may use it and for the parity status).
 *
 * Canonical math: DESIGN.md "Canonical math". There is no reference render code to cite
 * (SURVEY.md section 0); the stages follow SURVEY.md section 8(a) rows a9-a12 and the scene
 * generator spec of section 8(d). Built with -ffp-contract=off and -mfma: every fused
 * multiply-add is an explicit fmaf, every other operation is a single IEEE-754 binary32
 * operation, so this file and the HIP kernels evaluate identical expressions.
 */
#include "srt_oracle.h"

#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

/* ---- scene file: 80-byte header, then n*9 vertex floats, n*3 albedo floats ---------- */
int srto_scene_load(const char* path, srto_scene* out) {
    unsigned char head[80];
    uint32_t version;
    uint64_t n;
    FILE* f;
    memset(out, 0, sizeof(*out));
    f = fopen(path, "rb");
    if (!f) return -1;
    if (fread(head, 1, sizeof(head), f) != sizeof(head) || memcmp(head, "SRTSCN01", 8) != 0) {
        fclose(f);
        return -2;
    }
    memcpy(&version, head + 8, 4);
    memcpy(&n, head + 16, 8);
    if (version != 1 || n == 0 || n > (1ull << 31)) {
        fclose(f);
        return -3;
    }
    memcpy(out->camera, head + 24, 10 * sizeof(float));
    memcpy(out->background, head + 64, 3 * sizeof(float));
    out->n = (size_t)n;
    out->vertices = (float*)malloc(out->n * 9 * sizeof(float));
    out->albedo = (float*)malloc(out->n * 3 * sizeof(float));
    if (!out->vertices || !out->albedo || fread(out->vertices, sizeof(float), out->n * 9, f) != out->n * 9 ||
        fread(out->albedo, sizeof(float), out->n * 3, f) != out->n * 3) {
        fclose(f);
        srto_scene_free(out);
        return -4;
    }
    fclose(f);
    return 0;
}

void srto_scene_free(srto_scene* s) {
    free(s->vertices);
    free(s->albedo);
    s->vertices = NULL;
    s->albedo = NULL;
    s->n = 0;
}

/* ---- camera frame (double, rounded once) -------------------------------------------- */
void srto_frame(const float cam[10], size_t width, size_t height, float out[12]) {
    double f[3], r[3], u[3], up[3], len, half_h, half_w;
    int k;
    for (k = 0; k < 3; ++k) f[k] = (double)cam[3 + k] - (double)cam[k];
    len = sqrt(f[0] * f[0] + f[1] * f[1] + f[2] * f[2]);
    for (k = 0; k < 3; ++k) f[k] /= len;
    for (k = 0; k < 3; ++k) up[k] = cam[6 + k];
    r[0] = f[1] * up[2] - f[2] * up[1];
    r[1] = f[2] * up[0] - f[0] * up[2];
    r[2] = f[0] * up[1] - f[1] * up[0];
    len = sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]);
    for (k = 0; k < 3; ++k) r[k] /= len;
    u[0] = r[1] * f[2] - r[2] * f[1];
    u[1] = r[2] * f[0] - r[0] * f[2];
    u[2] = r[0] * f[1] - r[1] * f[0];
    half_h = tan((double)cam[9] * 3.14159265358979323846 / 360.0);
    half_w = half_h * (double)width / (double)height;
    for (k = 0; k < 3; ++k) {
        out[k] = cam[k];
        out[3 + k] = (float)(f[k] - half_w * r[k] + half_h * u[k]);
        out[6 + k] = (float)(2.0 * half_w * r[k]);
        out[9 + k] = (float)(-2.0 * half_h * u[k]);
    }
}

/* ---- float helpers: fixed evaluation order ------------------------------------------ */
static float dot3(const float* a, const float* b) { return fmaf(a[2], b[2], fmaf(a[1], b[1], a[0] * b[0])); }

static void cross3(const float* a, const float* b, float* c) {
    c[0] = a[1] * b[2] - a[2] * b[1];
    c[1] = a[2] * b[0] - a[0] * b[2];
    c[2] = a[0] * b[1] - a[1] * b[0];
}

/* ---- stage 1: edge records ---------------------------------------------------------- */
void srto_prepare(const float* vertices, size_t n, const float frame[12], float* edges) {
    size_t i;
    for (i = 0; i < n; ++i) {
        const float* v = vertices + 9 * i;
        float* e = edges + 12 * i;
        float a[3], b[3], c[3], nrm[3][3], vol;
        int k, j;
        for (k = 0; k < 3; ++k) {
            a[k] = v[k] - frame[k];
            b[k] = v[3 + k] - frame[k];
            c[k] = v[6 + k] - frame[k];
        }
        cross3(b, c, nrm[0]); /* edge opposite vertex 0 */
        cross3(c, a, nrm[1]);
        cross3(a, b, nrm[2]);
        vol = dot3(a, nrm[0]); /* 6 x signed volume of (eye, v0, v1, v2) */
        e[10] = 0.f;
        e[11] = 0.f;
        if (!(isfinite(vol) && vol != 0.f)) {
            for (k = 0; k < 10; ++k) e[k] = NAN;
            continue;
        }
        if (vol < 0.f) {
            for (j = 0; j < 3; ++j)
                for (k = 0; k < 3; ++k) nrm[j][k] = -nrm[j][k];
            vol = -vol;
        }
        for (j = 0; j < 3; ++j) {
            e[3 * j + 0] = dot3(nrm[j], frame + 3);
            e[3 * j + 1] = dot3(nrm[j], frame + 6);
            e[3 * j + 2] = dot3(nrm[j], frame + 9);
        }
        e[9] = vol;
    }
}

/* ---- stage 2: brute-force closest hit ------------------------------------------------ */
long srto_closest_hit(const float* edges, size_t n, float fx, float fy, float* t_out, float* det_out) {
    long best = -1;
    float best_t = INFINITY, best_det = 0.f;
    size_t i;
    for (i = 0; i < n; ++i) {
        const float* e = edges + 12 * i;
        const float ea = fmaf(fy, e[2], fmaf(fx, e[1], e[0]));
        const float eb = fmaf(fy, e[5], fmaf(fx, e[4], e[3]));
        const float ec = fmaf(fy, e[8], fmaf(fx, e[7], e[6]));
        /* non-short-circuit &: one rarely-taken branch instead of three unpredictable ones */
        if ((ea >= 0.f) & (eb >= 0.f) & (ec >= 0.f)) {
            const float det = (ea + eb) + ec;
            if (det > 0.f) {
                const float t = e[9] / det;
                if (t < best_t) { /* strict: the lowest id wins a tie */
                    best_t = t;
                    best_det = det;
                    best = (long)i;
                }
            }
        }
    }
    if (best >= 0) {
        if (t_out) *t_out = best_t;
        if (det_out) *det_out = best_det;
    }
    return best;
}

void srto_pixel_position(size_t x, size_t y, float sx, float sy, size_t width, size_t height, float* fx,
                         float* fy) {
    *fx = ((float)x + sx) / (float)width;
    *fy = ((float)y + sy) / (float)height;
}

/* ---- stage 3: shade ------------------------------------------------------------------ */
static void shade(const srto_scene* s, const float frame[12], long id, float fx, float fy, float* px) {
    float d[3], e1[3], e2[3], nrm[3], cosv;
    const float* v;
    const float* alb;
    int k;
    if (id < 0) {
        px[0] = s->background[0];
        px[1] = s->background[1];
        px[2] = s->background[2];
        px[3] = -1.f;
        return;
    }
    for (k = 0; k < 3; ++k) d[k] = fmaf(fy, frame[9 + k], fmaf(fx, frame[6 + k], frame[3 + k]));
    v = s->vertices + 9 * (size_t)id;
    for (k = 0; k < 3; ++k) {
        e1[k] = v[3 + k] - v[k];
        e2[k] = v[6 + k] - v[k];
    }
    cross3(e1, e2, nrm);
    cosv = fminf(fabsf(dot3(nrm, d)) / (sqrtf(dot3(nrm, nrm)) * sqrtf(dot3(d, d))), 1.f);
    alb = s->albedo + 3 * (size_t)id;
    px[0] = alb[0] * cosv;
    px[1] = alb[1] * cosv;
    px[2] = alb[2] * cosv;
    px[3] = (float)id;
}

int srto_threads(int threads) {
#ifdef _OPENMP
    return threads > 0 ? threads : omp_get_max_threads();
#else
    (void)threads;
    return 1;
#endif
}

size_t srto_render(const srto_scene* s, const float* offsets, size_t width, size_t height, size_t row_begin,
                   size_t row_count, size_t row_step, int threads, float* rgba) {
    float frame[12];
    float* edges;
    long r, rows;
    if (row_step == 0) row_step = 1;
    srto_frame(s->camera, width, height, frame);
    edges = (float*)malloc(s->n * 12 * sizeof(float));
    if (!edges) return 0;
    srto_prepare(s->vertices, s->n, frame, edges);
    rows = (long)((row_count + row_step - 1) / row_step);
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(srto_threads(threads))
#endif
    for (r = 0; r < rows; ++r) {
        const size_t y = row_begin + (size_t)r * row_step;
        size_t x;
        for (x = 0; x < width; ++x) {
            const float* o = offsets + 2 * (y * width + x);
            float fx, fy;
            long id;
            srto_pixel_position(x, y, o[0], o[1], width, height, &fx, &fy);
            id = srto_closest_hit(edges, s->n, fx, fy, NULL, NULL);
            shade(s, frame, id, fx, fy, rgba + 4 * (y * width + x));
        }
    }
    free(edges);
    return (size_t)rows;
}

/* Stage 3 alone (deferred shading, the multi-GPU band path): shade rows [row_begin, row_begin +
 * row_count) from hit ids (H x W, -1 = miss) and the offsets; same expressions as srto_render. */
void srto_shade(const srto_scene* s, const float* offsets, const int* ids, size_t width, size_t height,
                size_t row_begin, size_t row_count, float* rgba) {
    float frame[12];
    size_t y, x;
    srto_frame(s->camera, width, height, frame);
    for (y = row_begin; y < row_begin + row_count; ++y) {
        for (x = 0; x < width; ++x) {
            const float* o = offsets + 2 * (y * width + x);
            float fx, fy;
            srto_pixel_position(x, y, o[0], o[1], width, height, &fx, &fy);
            shade(s, frame, (long)ids[y * width + x], fx, fy, rgba + 4 * (y * width + x));
        }
    }
}
