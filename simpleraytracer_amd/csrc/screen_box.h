// Screen box of an edge record in float arithmetic with proven error bounds: the fast path of
// render.hip ScreenBox (the record pass's double-precision solve; DESIGN.md section 5 "Screen
// box"). Host and device share it (cpu_render.cpp, the host self-test srtScreenBoxHost).
//
// The box must contain every (fx, fy) with |fx|, |fy| <= F (F = kScreenBoxRange) at which the
// float test E_k = fma(fy, cy_k, fma(fx, cx_k, c0_k)) >= 0 passes for all three edges k. Such a
// point satisfies c0_k + S_k + cx_k fx + cy_k fy >= 0 in exact reals, S_k = 2^-24 (|c0_k| +
// F |cx_k|) + 2^-120 (the ScreenBox derivation). This routine:
//  1. computes a slack s_k >= S_k (below) and keeps the shifted constant c0_k + s_k as the
//     unevaluated pair (c0_k, s_k): rounding c0_k + s_k to one float would move the line by up to
//     an ulp of c0_k -- the size of the slack itself, which at a sharp corner of a small triangle
//     moves the corner by ~1e-4 (measured) --, so the region {c0_k + s_k + cx_k fx + cy_k fy >= 0}
//     contains the exact one;
//  2. decides whether the three gradients positively span the plane from the signs of the
//     determinants d = gx_i gy_j - gy_i gx_j, each computed by Kahan's FMA algorithm for ab - cd,
//     whose relative error is at most 2u (u = 2^-24; Jeannerod, Louvet, Muller 2013) -- so the
//     signs are exact;
//  3. solves each corner (the intersection of two shifted lines): numerator N = N1 + N2 with
//     N1 = c0_j gy_i - c0_i gy_j by Kahan's algorithm (2u relative) and the small slack term
//     N2 = s_j gy_i - s_i gy_j in plain float (3u of T2 = |s_j gy_i| + |s_i gy_j|), then one
//     reciprocal (v_rcp_f32: <= 1 ulp, 2u relative) and one product: |x^ - x| <= 8u |x| +
//     6u T2 / |d| to first order;
//  4. pads each corner by 2^-18 |x^| (64u) + 2^-20 T2 |1/d^| + 2^-80 and rounds to nearest:
//     lo <= x <= hi.
// Valid without underflow or overflow: every nonzero coefficient in [2^-40, 2^30] (c0: up to
// 2^30; gradients [2^-30, 2^30]), every |d| >= 2^-60, so the products of step 3 lie in [2^-70,
// 2^60] and corners below 2^122 (the slack products may underflow: absolute error <= 2^-148,
// times |1/d| <= 2^60, inside the 2^-80 pad). Otherwise (or for NaN / infinite inputs) it
// returns false and the caller takes the double solve, which handles every record.
//
// Step 1: t = fl(F |cx| + |c0|) >= (F |cx| + |c0|)(1 - u); s = fl((1 + 2^-20) 2^-24 t +
// 1.0625 * 2^-120) >= S' (1 - u)^2 (1 + 16u) + 2^-120 (1 - u) 1.0625 >= S' + 2^-120 = S, with
// S' = 2^-24 (|c0| + F |cx|).
#pragma once

#include <hip/hip_runtime.h>

#include <cmath>

namespace srt {

// a b - c d, relative error <= 2u (no underflow / overflow).
__host__ __device__ inline float KahanDiffOfProducts(float a, float b, float c, float d) {
    const float w = c * d;
    const float e = std::fmaf(-c, d, w);  // w - c d, exact
    const float f = std::fmaf(a, b, -w);
    return f + e;
}

__host__ __device__ inline float ApproxRcp(float d) {
#if defined(__HIP_DEVICE_COMPILE__)
    return __builtin_amdgcn_rcpf(d);  // <= 1 ulp
#else
    return 1.0f / d;
#endif
}

__host__ __device__ inline bool GradientInRange(float v) {
    const float a = std::fabs(v);
    return v == 0.f || (a >= 0x1p-30f && a <= 0x1p30f);  // NaN: false
}
__host__ __device__ inline bool ConstantInRange(float v) {
    const float a = std::fabs(v);
    return v == 0.f || (a >= 0x1p-40f && a <= 0x1p30f);  // NaN: false
}

// The solve in two halves sharing one setup, so a caller that may discard the record after its
// y-extent (a band's record pass: DESIGN.md section 5) skips the x half: ScreenBoxFast is exactly
// Setup, then Y, then X, the same operations on the same values.
struct BoxSolve {
    float gx[3], gy[3], c0[3], s[3];
    float r[3];    // ApproxRcp of the corner determinants (corner v: lines (v + 1) % 3, (v + 2) % 3)
    bool ok;       // the float solve applies (else the double one)
    bool spans;    // the gradients positively span the plane (else the box is unbounded)
};

__host__ __device__ inline void ScreenBoxSetup(const float c[9], float range, BoxSolve& b) {
    b.ok = true;
    for (int e = 0; e < 3; ++e) {
        b.c0[e] = c[3 * e];
        b.gx[e] = c[3 * e + 1];
        b.gy[e] = c[3 * e + 2];
        const float t = std::fmaf(range, std::fabs(b.gx[e]), std::fabs(b.c0[e]));
        b.s[e] = std::fmaf(0x1.00001p-24f, t, 0x1.1p-120f);
        b.ok = b.ok && ConstantInRange(b.c0[e]) && GradientInRange(b.gx[e]) && GradientInRange(b.gy[e]);
    }
    if (!b.ok) {
        b.spans = false;
        return;
    }
    const float dAB = KahanDiffOfProducts(b.gx[0], b.gy[1], b.gy[0], b.gx[1]);
    const float dBC = KahanDiffOfProducts(b.gx[1], b.gy[2], b.gy[1], b.gx[2]);
    const float dCA = KahanDiffOfProducts(b.gx[2], b.gy[0], b.gy[2], b.gx[0]);
    b.spans = (dAB > 0.f && dBC > 0.f && dCA > 0.f) || (dAB < 0.f && dBC < 0.f && dCA < 0.f);
    const float dv[3] = {dBC, dCA, dAB};
    for (int v = 0; v < 3; ++v) {
        b.ok = b.ok && (!b.spans || std::fabs(dv[v]) >= 0x1p-60f);
        b.r[v] = ApproxRcp(dv[v]);
    }
}

// y = (gx_j k_i - gx_i k_j) / d over the three corners (k = c0 + s), padded: (ylo, yhi). Needs
// b.ok && b.spans.
__host__ __device__ inline void ScreenBoxY(const BoxSolve& b, float& ylo, float& yhi) {
    ylo = INFINITY;
    yhi = -INFINITY;
    for (int v = 0; v < 3; ++v) {
        const int i = (v + 1) % 3, j = (v + 2) % 3;
        const float r = b.r[v], ar = std::fabs(r);
        const float sy1 = b.gx[j] * b.s[i], sy2 = b.gx[i] * b.s[j];
        const float ny = KahanDiffOfProducts(b.gx[j], b.c0[i], b.gx[i], b.c0[j]) + (sy1 - sy2);
        const float y = ny * r;
        const float py = std::fmaf(0x1p-18f, std::fabs(y), std::fmaf(0x1p-20f * ar, std::fabs(sy1) + std::fabs(sy2), 0x1p-80f));
        ylo = std::fmin(ylo, y - py);
        yhi = std::fmax(yhi, y + py);
    }
}

// x = (k_j gy_i - k_i gy_j) / d over the three corners, padded: (xlo, xhi). Needs b.ok && b.spans.
__host__ __device__ inline void ScreenBoxX(const BoxSolve& b, float& xlo, float& xhi) {
    xlo = INFINITY;
    xhi = -INFINITY;
    for (int v = 0; v < 3; ++v) {
        const int i = (v + 1) % 3, j = (v + 2) % 3;
        const float r = b.r[v], ar = std::fabs(r);
        const float sx1 = b.s[j] * b.gy[i], sx2 = b.s[i] * b.gy[j];
        const float nx = KahanDiffOfProducts(b.c0[j], b.gy[i], b.c0[i], b.gy[j]) + (sx1 - sx2);
        const float x = nx * r;
        const float px = std::fmaf(0x1p-18f, std::fabs(x), std::fmaf(0x1p-20f * ar, std::fabs(sx1) + std::fabs(sx2), 0x1p-80f));
        xlo = std::fmin(xlo, x - px);
        xhi = std::fmax(xhi, x + px);
    }
}

// c = (c0A, cxA, cyA, c0B, cxB, cyB, c0C, cxC, cyC); range = F. true: *box = (xlo, xhi, ylo, yhi),
// possibly unbounded (the gradients do not span the plane); false: use the double solve.
__host__ __device__ inline bool ScreenBoxFast(const float c[9], float range, float box[4]) {
    BoxSolve b;
    ScreenBoxSetup(c, range, b);
    if (!b.ok) {
        return false;
    }
    if (!b.spans) {
        box[0] = -INFINITY;
        box[1] = INFINITY;
        box[2] = -INFINITY;
        box[3] = INFINITY;
        return true;
    }
    ScreenBoxY(b, box[2], box[3]);
    ScreenBoxX(b, box[0], box[1]);
    return true;
}

}  // namespace srt
