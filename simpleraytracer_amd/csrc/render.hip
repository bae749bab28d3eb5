// MI355X (gfx950) render kernels: edge-record preparation and the brute-force closest-hit
// trace. The reference has no render code; this file implements the
// north_star stages (a9)-(a12) of SURVEY.md section 8(a) from the canonical math in
// DESIGN.md. Built with -ffp-contract=off: every fused multiply-add below is an explicit
// fmaf, so CPU (oracle/srt_oracle.c) and GPU evaluate bit-identical float expressions.
#include "render.h"

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>

namespace srt {

#ifdef SRT_DIAG
// Diagnostic build only (make diag): per-block phase cycle counts of the cull kernel.
// [block][0] stream cycles, [1] gather cycles, [2] filter+walk cycles, [3] block survivors,
// [4] wave-0 survivors walked, [5] flush batches, [6] total cycles, [7] unused.
constexpr int kDiagBlocks = 65536;
__device__ unsigned long long g_srt_diag[kDiagBlocks][8];
#define SRT_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
#else
#define SRT_STAMP(v)
#endif

namespace {

constexpr int kWave = 64;
constexpr int kLdsWaves = 4;     // waves per block in the LDS variant
constexpr int kRowsPerLane = 8;  // rays per lane (LDS / scalar variants): one column, 8 rows

struct TraceParams {
    const float4* __restrict__ edges;
    const float4* __restrict__ screen_boxes;
    const uint2* __restrict__ qboxes;
    const float* __restrict__ vertices;
    const float* __restrict__ albedo;
    const float2* __restrict__ offsets;
    float4* __restrict__ out;
    unsigned n_pad;   // records in the edge buffer (multiple of kPadTriangles)
    unsigned n_tiles; // tiles holding at least one real record (>= 1)
    int width;
    int row_count;
    int row_begin;
    int allow_raster;  // cull variant: raster walk for uniform-offset tiles (env SRT_CULL_RASTER=0 disables)
    const unsigned* __restrict__ bin_lists;   // cull variant: per super-tile candidate ids (BinKernel)
    const unsigned* __restrict__ bin_counts;  // null: stream every record
    unsigned bin_capacity;
    unsigned chunk_ids;                          // cull: list ids per block of a split tile
    unsigned long long* __restrict__ tile_keys;  // cull, split tiles: per-pixel (t, id) keys (band)
    unsigned* __restrict__ tile_done;            // cull, split tiles: finished blocks per tile
    float wf;
    float hf;
    float base[3];
    float du[3];
    float dv[3];
    float bg[3];
};

struct PrepareParams {
    const float* __restrict__ vertices;
    float4* __restrict__ edges;
    float4* __restrict__ screen_boxes;
    uint2* __restrict__ qboxes;
    unsigned n;
    unsigned n_pad;
    float origin[3];
    float base[3];
    float du[3];
    float dv[3];
};

// One edge record as the trace kernels consume it.
struct Record {
    float c0A, cxA, cyA, c0B, cxB, cyB, c0C, cxC, cyC;
};

__device__ __forceinline__ float Dot3(float ax, float ay, float az, float bx, float by, float bz) {
    return fmaf(az, bz, fmaf(ay, by, ax * bx));
}

__device__ __forceinline__ void Cross3(float ax, float ay, float az, float bx, float by, float bz, float& cx,
                                       float& cy, float& cz) {
    cx = ay * bz - az * by;
    cy = az * bx - ax * bz;
    cz = ax * by - ay * bx;
}

// Plane addresses of record j of the tile starting at `tile` (render.h "tile-planar").
__device__ __forceinline__ const float* Plane2(const float4* tile) {
    return reinterpret_cast<const float*>(tile + 2 * kTileTriangles);
}
__device__ __forceinline__ const float* Plane3(const float4* tile) {
    return reinterpret_cast<const float*>(tile + 2 * kTileTriangles) + kTileTriangles;
}

// Screen box of a record: an (fx, fy) box containing every ray position with |fx| <= F
// (F = kScreenBoxRange) at which the float test E_k = fma(fy, cy_k, fma(fx, cx_k, c0_k)) >= 0
// can pass for all three edges. Derivation (DESIGN.md "Screen box"): with g = fl(fx cx + c0)
// = (fx cx + c0)(1 + d), |d| <= 2^-24, plus an absolute term for subnormal results, the
// outer fma only rounds (sign-preserving, -0 passes), so a pass implies
//     c0 + cx fx + cy fy >= -s,   s = 2^-24 (|c0| + F |cx|) + 2^-120   (exact reals).
// If the three gradients (cx_k, cy_k) positively span the plane (exact sign tests in double:
// the products of two floats are exact), the region {c0_k + s_k + cx_k fx + cy_k fy >= 0} is
// bounded: the triangle whose corners are the pairwise line intersections (empty otherwise,
// which any box covers). Corners are solved in double, padded for double rounding and
// rounded outward to float. Otherwise the box is unbounded (never culls).
__device__ __forceinline__ float DownF(double v) { return __double2float_rd(v); }
__device__ __forceinline__ float UpF(double v) { return __double2float_ru(v); }

__device__ float4 ScreenBox(const float c[9]) {
    const float inf = __builtin_inff();
    const float4 unbounded = make_float4(-inf, inf, -inf, inf);
    double gx[3], gy[3], k[3];
    for (int e = 0; e < 3; ++e) {
        const double c0 = c[3 * e], cx = c[3 * e + 1], cy = c[3 * e + 2];
        if (!(fabs(c0) < 1e30 && fabs(cx) < 1e30 && fabs(cy) < 1e30)) {
            return unbounded;
        }
        gx[e] = cx;
        gy[e] = cy;
        const double slack = (0x1p-24 * (fabs(c0) + kScreenBoxRange * fabs(cx)) + 0x1p-120) * (1.0 + 1e-12);
        k[e] = c0 + slack;  // shifted constant; |error| of this sum is covered by the pad below
    }
    const double dAB = gx[0] * gy[1] - gy[0] * gx[1];
    const double dBC = gx[1] * gy[2] - gy[1] * gx[2];
    const double dCA = gx[2] * gy[0] - gy[2] * gx[0];
    const bool spans = (dAB > 0 && dBC > 0 && dCA > 0) || (dAB < 0 && dBC < 0 && dCA < 0);
    if (!spans) {
        return unbounded;
    }
    double xlo = 1e300, xhi = -1e300, ylo = 1e300, yhi = -1e300;
    for (int v = 0; v < 3; ++v) {
        const int i = (v + 1) % 3, j = (v + 2) % 3;  // corner opposite edge v: lines i and j
        const double d = gx[i] * gy[j] - gy[i] * gx[j];
        const double tx1 = -k[i] * gy[j], tx2 = k[j] * gy[i];
        const double ty1 = -gx[i] * k[j], ty2 = gx[j] * k[i];
        const double x = (tx1 + tx2) / d, y = (ty1 + ty2) / d;
        const double ad = fabs(d);
        const double px = 1e-12 * ((fabs(tx1) + fabs(tx2)) / ad + fabs(x)) + 1e-300;
        const double py = 1e-12 * ((fabs(ty1) + fabs(ty2)) / ad + fabs(y)) + 1e-300;
        xlo = fmin(xlo, x - px);
        xhi = fmax(xhi, x + px);
        ylo = fmin(ylo, y - py);
        yhi = fmax(yhi, y + py);
    }
    if (!(xlo <= xhi && ylo <= yhi)) {
        return unbounded;
    }
    return make_float4(DownF(xlo), UpF(xhi), DownF(ylo), UpF(yhi));
}

// int16 fixed point of a screen-box coordinate, rounded down (lo) or up (hi), clamped to
// [-32767, 32767]; the map is monotone, so an overlap of two real boxes is an overlap of
// their quantized boxes. (Clamping lo upward at -32767 only matters for coordinates below
// -8, where no ray box the screen boxes apply to, |fx|, |fy| <= 4, reaches.)
__device__ __forceinline__ int QuantLo(float v) {
    const float q = floorf(v * kQuantScale);  // exact scaling (power of two); NaN -> lowest
    return q >= 32767.f ? 32767 : (q >= -32767.f ? static_cast<int>(q) : -32767);
}
__device__ __forceinline__ int QuantHi(float v) {
    const float q = ceilf(v * kQuantScale);
    return q <= -32767.f ? -32767 : (q <= 32767.f ? static_cast<int>(q) : 32767);
}
__device__ __forceinline__ unsigned PackI16(int low, int high) {
    return (static_cast<unsigned>(low) & 0xFFFFu) | (static_cast<unsigned>(high) << 16);
}

// One thread per triangle: origin-relative edge normals nA = B x C, nB = C x A, nC = A x B
// (A, B, C = vertices - eye), signed volume vol = A . nA, orientation normalised so vol > 0,
// then each normal projected onto the affine ray frame: E(fx, fy) = n . (base + fx du + fy dv).
__global__ __launch_bounds__(256) void PrepareKernel(PrepareParams p) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n_pad) {
        return;
    }
    float4* tile = p.edges + static_cast<size_t>(i / kTileTriangles) * kTileFloat4;
    const unsigned j = i % kTileTriangles;
    float* p2 = reinterpret_cast<float*>(tile + 2 * kTileTriangles);
    float* p3 = p2 + kTileTriangles;
    const float qnan = __builtin_nanf("");
    bool disabled = i >= p.n;
    float c[9];
    float vol = qnan;
    if (!disabled) {
        const float* v = p.vertices + 9ull * i;
        const float ax = v[0] - p.origin[0], ay = v[1] - p.origin[1], az = v[2] - p.origin[2];
        const float bx = v[3] - p.origin[0], by = v[4] - p.origin[1], bz = v[5] - p.origin[2];
        const float cx = v[6] - p.origin[0], cy = v[7] - p.origin[1], cz = v[8] - p.origin[2];
        float n[9];
        Cross3(bx, by, bz, cx, cy, cz, n[0], n[1], n[2]);
        Cross3(cx, cy, cz, ax, ay, az, n[3], n[4], n[5]);
        Cross3(ax, ay, az, bx, by, bz, n[6], n[7], n[8]);
        vol = Dot3(ax, ay, az, n[0], n[1], n[2]);
        disabled = !(std::isfinite(vol) && vol != 0.f);
        if (!disabled) {
            if (vol < 0.f) {
#pragma unroll
                for (int k = 0; k < 9; ++k) {
                    n[k] = -n[k];
                }
                vol = -vol;
            }
#pragma unroll
            for (int e = 0; e < 3; ++e) {
                const float nx = n[3 * e], ny = n[3 * e + 1], nz = n[3 * e + 2];
                c[3 * e + 0] = Dot3(nx, ny, nz, p.base[0], p.base[1], p.base[2]);
                c[3 * e + 1] = Dot3(nx, ny, nz, p.du[0], p.du[1], p.du[2]);
                c[3 * e + 2] = Dot3(nx, ny, nz, p.dv[0], p.dv[1], p.dv[2]);
            }
        }
    }
    if (disabled) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            c[k] = qnan;
        }
        vol = qnan;
    }
    tile[j] = make_float4(c[0], c[1], c[2], c[3]);
    tile[kTileTriangles + j] = make_float4(c[4], c[5], c[6], c[7]);
    p2[j] = c[8];
    p3[j] = vol;
    // Disabled records: an empty box (culled by every ray box the screen boxes apply to).
    const float4 sb = disabled ? make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff())
                               : ScreenBox(c);
    p.screen_boxes[i] = sb;
    // Stored as (hi, -lo) pairs so the cull test is one saturating packed add per axis.
    p.qboxes[i] = make_uint2(PackI16(QuantHi(sb.y), -QuantLo(sb.x)), PackI16(QuantHi(sb.w), -QuantLo(sb.z)));
}

// Per-lane ray state: R rays sharing one image column.
template <int R>
struct Rays {
    float fx[R];
    float fy[R];
    float bt[R];  // closest t so far (+inf = none)
    int bi[R];    // closest triangle id (-1 = miss)
};

// Axis-aligned box in image-position space (fx, fy) containing a set of rays.
struct Box {
    float xlo, xhi, ylo, yhi;
};

// Conservative rejection of a record for every ray whose (fx, fy) lies in the box.
// E_k = fma(fy, cy, fma(fx, cx, c0)) is monotone in fx (sign of cx) and in fy (sign of cy),
// because a correctly rounded fma is monotone in each argument; so its maximum over the box
// is attained at the corner picked by the signs, and a ray in the box can pass the exact
// test (all E_k >= 0) only if no corner value is < 0. NaN corner values never reject.
// Exact: a rejected record fails the exact test for every ray of the box, bit for bit.
__device__ __forceinline__ bool BoxMayHit(const Box& b, const Record& q) {
    const float eA = fmaf(q.cyA >= 0.f ? b.yhi : b.ylo, q.cyA, fmaf(q.cxA >= 0.f ? b.xhi : b.xlo, q.cxA, q.c0A));
    const float eB = fmaf(q.cyB >= 0.f ? b.yhi : b.ylo, q.cyB, fmaf(q.cxB >= 0.f ? b.xhi : b.xlo, q.cxB, q.c0B));
    const float eC = fmaf(q.cyC >= 0.f ? b.yhi : b.ylo, q.cyC, fmaf(q.cxC >= 0.f ? b.xhi : b.xlo, q.cxC, q.c0C));
    return !(eA < 0.f || eB < 0.f || eC < 0.f);
}

// Test one triangle's edge record against the lane's R rays (brute force: every ray).
//   hot path:  E_A, E_B, E_C for every ray, candidate iff min(E) >= 0 for some ray
//              (one branch per triangle per wave; candidates are rare)
//   slow path: exact test per ray: all E >= 0, det = (E_A + E_B) + E_C > 0, t = vol / det,
//              strict t < best keeps the lowest id on ties (triangles arrive in id order).
// SHARED: every ray of the lane has the same fx bit pattern, so fma(fx, cx, c0) is one
// value per edge (common-subexpression elimination; the result is bit-identical).
template <int R, bool SHARED>
__device__ __forceinline__ void TestTriangle(Rays<R>& s, const Record& q, unsigned id, const float* vol_ptr) {
    float gA[R], gB[R], gC[R];
    if constexpr (SHARED) {
        const float a = fmaf(s.fx[0], q.cxA, q.c0A), b = fmaf(s.fx[0], q.cxB, q.c0B),
                    c = fmaf(s.fx[0], q.cxC, q.c0C);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gA[r] = a;
            gB[r] = b;
            gC[r] = c;
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gA[r] = fmaf(s.fx[r], q.cxA, q.c0A);
            gB[r] = fmaf(s.fx[r], q.cxB, q.c0B);
            gC[r] = fmaf(s.fx[r], q.cxC, q.c0C);
        }
    }
    float m[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float eA = fmaf(s.fy[r], q.cyA, gA[r]);
        const float eB = fmaf(s.fy[r], q.cyB, gB[r]);
        const float eC = fmaf(s.fy[r], q.cyC, gC[r]);
        m[r] = fminf(fminf(eA, eB), eC);
    }
    // max-tree over the rays (NaN edges from disabled records drop out of fmaxf)
#pragma unroll
    for (int w = 1; w < R; w *= 2) {
#pragma unroll
        for (int r = 0; r + w < R; r += 2 * w) {
            m[r] = fmaxf(m[r], m[r + w]);
        }
    }
    if (m[0] >= 0.f) {
        const float vol = *vol_ptr;
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const float eA = fmaf(s.fy[r], q.cyA, gA[r]);
            const float eB = fmaf(s.fy[r], q.cyB, gB[r]);
            const float eC = fmaf(s.fy[r], q.cyC, gC[r]);
            if (eA >= 0.f && eB >= 0.f && eC >= 0.f) {
                const float det = (eA + eB) + eC;
                if (det > 0.f) {
                    const float t = vol / det;
                    if (t < s.bt[r]) {
                        s.bt[r] = t;
                        s.bi[r] = static_cast<int>(id);
                    }
                }
            }
        }
    }
}

// Ray generation: lane owns column x, rows y0..y0+R-1 of the band (clamped for edge lanes;
// clamped lanes compute but never store). Returns whether all R rays share fx's bit
// pattern; `box` receives the rays' (fx, fy) bounding box (NaN positions drop out: a ray
// with a NaN position fails every test).
template <int R>
__device__ __forceinline__ bool GenerateRays(const TraceParams& p, int x, int y0, Rays<R>& s, Box& box) {
    const int xc = min(x, p.width - 1);
    bool same = true;
    box = Box{__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()};
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int yc = min(y0 + r, p.row_count - 1);
        const float2 o = p.offsets[static_cast<size_t>(yc) * p.width + xc];
        s.fx[r] = (static_cast<float>(xc) + o.x) / p.wf;
        s.fy[r] = (static_cast<float>(p.row_begin + yc) + o.y) / p.hf;
        s.bt[r] = __builtin_inff();
        s.bi[r] = -1;
        same = same && (__float_as_uint(s.fx[r]) == __float_as_uint(s.fx[0]));
        box.xlo = fminf(box.xlo, s.fx[r]);
        box.xhi = fmaxf(box.xhi, s.fx[r]);
        box.ylo = fminf(box.ylo, s.fy[r]);
        box.yhi = fmaxf(box.yhi, s.fy[r]);
    }
    return same;
}

// Shade + store: rgb = albedo * |cos(N, d)| for a hit, background for a miss; alpha carries
// float(tri_id) (exact for ids < 2^24), -1 for a miss.
template <int R>
__device__ __forceinline__ void ShadeAndStore(const TraceParams& p, int x, int y0, const Rays<R>& s) {
    if (x >= p.width) {
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int y = y0 + r;
        if (y >= p.row_count) {
            continue;
        }
        float4 o;
        const int id = s.bi[r];
        if (id >= 0) {
            const float fx = s.fx[r], fy = s.fy[r];
            const float dx = fmaf(fy, p.dv[0], fmaf(fx, p.du[0], p.base[0]));
            const float dy = fmaf(fy, p.dv[1], fmaf(fx, p.du[1], p.base[1]));
            const float dz = fmaf(fy, p.dv[2], fmaf(fx, p.du[2], p.base[2]));
            const float* v = p.vertices + 9ull * id;
            const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
            const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
            float nx, ny, nz;
            Cross3(e1x, e1y, e1z, e2x, e2y, e2z, nx, ny, nz);
            const float nd = Dot3(nx, ny, nz, dx, dy, dz);
            const float nn = Dot3(nx, ny, nz, nx, ny, nz);
            const float dd = Dot3(dx, dy, dz, dx, dy, dz);
            const float cosv = fminf(fabsf(nd) / (sqrtf(nn) * sqrtf(dd)), 1.f);
            const float* a = p.albedo + 3ull * id;
            o = make_float4(a[0] * cosv, a[1] * cosv, a[2] * cosv, static_cast<float>(id));
        } else {
            o = make_float4(p.bg[0], p.bg[1], p.bg[2], -1.f);
        }
        p.out[static_cast<size_t>(y) * p.width + x] = o;
    }
}

// ---------------------------------------------------------------------------------------
// Variant 0: LDS-tiled brute force. Block = 4 waves = 64 columns x 32 rows. Each 10 KiB
// tile of edge records is copied by the whole block into one half of a double-buffered LDS
// ring, then every wave walks it with broadcast LDS reads: every ray tests every record.
// One barrier per tile; the next tile's copy is in flight during the current one.
// ---------------------------------------------------------------------------------------
using LdsVoidPtr = __attribute__((address_space(3))) void*;

// Copy one 10 KiB tile global -> LDS with LDS-DMA (global_load_lds_dwordx4): 10 wave-
// instructions of 1 KiB, spread over the block's waves, no VGPR staging; the LDS image is
// the global image. Issued through inline asm so hipcc does not drain it with a vmcnt(0) in
// front of every ds_read of the tile being computed (cdna_hip_programming.md section 5
// "Pipelining across barriers"); completion is waited for by WaitTile().
__device__ __forceinline__ void StageTile(const float4* __restrict__ src, float4* dst) {
    constexpr int kChunks = kTileFloat4 / kWave;  // 10
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
#pragma unroll
    for (int k = 0; k < (kChunks + kLdsWaves - 1) / kLdsWaves; ++k) {
        const int c = wave + k * kLdsWaves;
        if (c < kChunks) {
            const int chunk = c * kWave;
            const float4* gsrc = src + chunk + lane;
            const unsigned lds_dst = __builtin_amdgcn_readfirstlane(
                static_cast<unsigned>(reinterpret_cast<size_t>((LdsVoidPtr)(void*)(dst + chunk))));
            unsigned keep;
            asm volatile(
                "s_mov_b32 %0, m0\n\t"
                "s_mov_b32 m0, %2\n\t"
                "s_nop 0\n\t"
                "global_load_lds_dwordx4 %1, off\n\t"
                "s_mov_b32 m0, %0"
                : "=&s"(keep)
                : "v"(gsrc), "s"(lds_dst)
                : "memory");
        }
    }
}

// Every wave's LDS-DMA done, then the block barrier makes the tile visible to all waves.
__device__ __forceinline__ void WaitTile() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

template <int R, bool SHARED>
__device__ __forceinline__ void WalkTilesLds(const TraceParams& p, float4* lds, Rays<R>& s) {
    const unsigned ntiles = p.n_tiles;
    StageTile(p.edges, lds);
    for (unsigned t = 0; t < ntiles; ++t) {
        const unsigned buf = t & 1u;
        WaitTile();  // tile t landed; every wave is done with tile t-1 (the buffer refilled next)
        if (t + 1 < ntiles) {
            StageTile(p.edges + static_cast<size_t>(t + 1) * kTileFloat4, lds + (buf ^ 1u) * kTileFloat4);
        }
        const float4* tile = lds + buf * kTileFloat4;
        const float* p2 = Plane2(tile);
        const float* p3 = Plane3(tile);
        const unsigned id0 = t * kTileTriangles;
#pragma unroll 2
        for (int j = 0; j < kTileTriangles; ++j) {
            const float4 q0 = tile[j];
            const float4 q1 = tile[kTileTriangles + j];
            const Record q{q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, p2[j]};
            TestTriangle<R, SHARED>(s, q, id0 + j, p3 + j);
        }
    }
}

__global__ __launch_bounds__(kWave * kLdsWaves) void TraceLdsKernel(TraceParams p) {
    // ONE __shared__ object: the double-buffered tile ring plus one flag word at the end
    // (a second LDS object next to LDS-DMA staging makes hipcc wait vmcnt(0) before every
    // ds_read; cdna_hip_programming.md section 5 trap 4(a)).
    __shared__ float4 lds[2 * kTileFloat4 + 1];
    constexpr int R = kRowsPerLane;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int x = blockIdx.x * kWave + lane;
    const int y0 = (blockIdx.y * kLdsWaves + wave) * R;
    Rays<R> s;
    Box box;
    const bool same = GenerateRays<R>(p, x, y0, s, box);
    // Block-uniform choice of loop body (both bodies hold the same barriers).
    unsigned* flag = reinterpret_cast<unsigned*>(lds + 2 * kTileFloat4);
    if (threadIdx.x == 0) {
        *flag = 1u;
    }
    __syncthreads();
    if (!__all(same) && lane == 0) {
        *flag = 0u;
    }
    __syncthreads();
    if (*flag != 0u) {
        WalkTilesLds<R, true>(p, lds, s);
    } else {
        WalkTilesLds<R, false>(p, lds, s);
    }
    ShadeAndStore<R>(p, x, y0, s);
}

// ---------------------------------------------------------------------------------------
// Variant 1: scalar stream. Block = 1 wave = 64 columns x 8 rows. The edge records are read
// with wave-uniform addresses, so they arrive through the scalar cache into SGPRs and feed
// the VALU FMAs directly; no LDS, no barriers, every wave independent.
// ---------------------------------------------------------------------------------------
template <int R, bool SHARED>
__device__ __forceinline__ void WalkScalar(const TraceParams& p, Rays<R>& s) {
    const unsigned ntiles = p.n_tiles;
    for (unsigned t = 0; t < ntiles; ++t) {
        const float4* tile = p.edges + static_cast<size_t>(t) * kTileFloat4;
        const float* p2 = Plane2(tile);
        const float* p3 = Plane3(tile);
#pragma unroll 4
        for (int j = 0; j < kTileTriangles; ++j) {
            const float4 q0 = tile[j];
            const float4 q1 = tile[kTileTriangles + j];
            const Record q{q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, p2[j]};
            TestTriangle<R, SHARED>(s, q, t * kTileTriangles + j, p3 + j);
        }
    }
}

__global__ __launch_bounds__(kWave) void TraceScalarKernel(TraceParams p) {
    constexpr int R = kRowsPerLane;
    const int x = blockIdx.x * kWave + static_cast<int>(threadIdx.x);
    const int y0 = blockIdx.y * R;
    Rays<R> s;
    Box box;
    const bool same = GenerateRays<R>(p, x, y0, s, box);
    if (__all(same)) {
        WalkScalar<R, true>(p, s);
    } else {
        WalkScalar<R, false>(p, s);
    }
    ShadeAndStore<R>(p, x, y0, s);
}

// ---------------------------------------------------------------------------------------
// Variant 2: hierarchical cull ("packet-frustum" brute force). Block = W waves; wave w owns
// 64 columns x R rows, the block 64 columns x W*R rows. Every record of the scene is still
// visited by every block, in three exact levels:
//   1. block: one lane per record streams the 8-B quantized screen boxes (PrepareKernel, "Screen
//      box"), G records per lane per step loaded one step ahead, and tests them against
//      the block's (fx, fy) box; the ids of survivors are appended (wave ballot + prefix
//      popcount) to the wave's LDS id list;
//   2. wave:  once the lists hold a batch (or at the end) the block gathers the survivors'
//      edge records into LDS; each wave tests them, one per lane, against its own box
//      (screen box + BoxMayHit) and ballots the result;
//   3. ray:   for every set bit, the exact per-ray test of all the wave's rays, keeping the
//      lexicographic (t, id) minimum (survivors arrive out of id order).
// Levels 1-2 only drop records that provably fail the exact test for every ray they cover,
// so the frame is bit-identical to the brute-force variants.
// ---------------------------------------------------------------------------------------
__device__ __forceinline__ Box WaveReduceBox(Box b) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        b.xlo = fminf(b.xlo, __shfl_xor(b.xlo, o));
        b.xhi = fmaxf(b.xhi, __shfl_xor(b.xhi, o));
        b.ylo = fminf(b.ylo, __shfl_xor(b.ylo, o));
        b.yhi = fmaxf(b.yhi, __shfl_xor(b.yhi, o));
    }
    return b;
}

// The screen boxes bound only rays with |fx|, |fy| <= kScreenBoxRange (PrepareKernel); a
// ray box reaching outside that square (or NaN) skips the screen-box test.
__device__ __forceinline__ bool ScreenBoxUsable(const Box& b) {
    return b.xlo >= -kScreenBoxRange && b.xhi <= kScreenBoxRange && b.ylo >= -kScreenBoxRange &&
           b.yhi <= kScreenBoxRange;
}

// Screen box (xlo, xhi, ylo, yhi) of a record overlaps the ray box.
__device__ __forceinline__ bool ScreenBoxOverlaps(const Box& b, const float4& sb) {
    return !(sb.y < b.xlo || sb.x > b.xhi || sb.w < b.ylo || sb.z > b.yhi);
}

// Quantized ray box for the streamed int16 screen boxes, as the per-axis constants of the
// packed test: a record's (hi, -lo) + (-box_lo, box_hi) = (hi - box_lo, box_hi - lo), and the
// boxes overlap iff no half is negative (v_pk_add_i16 with clamp: saturation keeps signs).
typedef short I16x2 __attribute__((ext_vector_type(2)));
struct QBox {
    unsigned x, y;
};
__device__ __forceinline__ QBox Quantize(const Box& b) {
    return QBox{PackI16(-QuantLo(b.xlo), QuantHi(b.xhi)), PackI16(-QuantLo(b.ylo), QuantHi(b.yhi))};
}
__device__ __forceinline__ bool QBoxOverlaps(const QBox& b, unsigned qx, unsigned qy) {
    const I16x2 sx = __builtin_elementwise_add_sat(__builtin_bit_cast(I16x2, qx), __builtin_bit_cast(I16x2, b.x));
    const I16x2 sy = __builtin_elementwise_add_sat(__builtin_bit_cast(I16x2, qy), __builtin_bit_cast(I16x2, b.y));
    return ((__builtin_bit_cast(unsigned, sx) | __builtin_bit_cast(unsigned, sy)) & 0x80008000u) == 0u;
}

// Exact test of one record against every ray of the lane (records in any order): the
// lexicographic minimum of (t, id) equals the ascending-id strict-< result of TestTriangle
// (smallest t; among equal t the lowest id).
template <int R, bool SHARED>
__device__ __forceinline__ void ExactTestAnyOrder(Rays<R>& s, const Record& q, float vol, int id) {
    float gA[R], gB[R], gC[R];
    if constexpr (SHARED) {
        const float a = fmaf(s.fx[0], q.cxA, q.c0A), b = fmaf(s.fx[0], q.cxB, q.c0B),
                    c = fmaf(s.fx[0], q.cxC, q.c0C);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gA[r] = a;
            gB[r] = b;
            gC[r] = c;
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gA[r] = fmaf(s.fx[r], q.cxA, q.c0A);
            gB[r] = fmaf(s.fx[r], q.cxB, q.c0B);
            gC[r] = fmaf(s.fx[r], q.cxC, q.c0C);
        }
    }
    float e[R][3];
    float m[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        e[r][0] = fmaf(s.fy[r], q.cyA, gA[r]);
        e[r][1] = fmaf(s.fy[r], q.cyB, gB[r]);
        e[r][2] = fmaf(s.fy[r], q.cyC, gC[r]);
        m[r] = fminf(fminf(e[r][0], e[r][1]), e[r][2]);
    }
    float mm = m[0];
#pragma unroll
    for (int r = 1; r < R; ++r) {
        mm = fmaxf(mm, m[r]);
    }
    if (mm >= 0.f) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            if (e[r][0] >= 0.f && e[r][1] >= 0.f && e[r][2] >= 0.f) {
                const float det = (e[r][0] + e[r][1]) + e[r][2];
                if (det > 0.f) {
                    const float t = vol / det;
                    if (t < s.bt[r] || (t == s.bt[r] && id < s.bi[r])) {
                        s.bt[r] = t;
                        s.bi[r] = id;
                    }
                }
            }
        }
    }
}

// Loads record `id`'s edge planes from the tile-planar buffer.
__device__ __forceinline__ void LoadRecord(const float4* __restrict__ edges, unsigned id, float4& p0, float4& p1,
                                           float& cyC, float& vol) {
    const float4* tile = edges + static_cast<size_t>(id / kTileTriangles) * kTileFloat4;
    const unsigned j = id % kTileTriangles;
    p0 = tile[j];
    p1 = tile[kTileTriangles + j];
    cyC = Plane2(tile)[j];
    vol = Plane3(tile)[j];
}

// Cull tile = one trace block: 64 columns x 32 rows of rays, W waves (4, 8 or 16) of 64 x R
// rays, R = 32 / W rays per lane. Constants that depend on W live in CullShape<W>.
constexpr int kTileRows = 32;
constexpr int kStreamStep = 2048;  // FULL stream: records per block per step
constexpr int kListG = 4;          // LIST stream: ids per lane per step
static_assert(kPadTriangles % kStreamStep == 0, "a stream step must cover whole pad units");

template <int W>
struct CullShape {
    static constexpr int kR = kTileRows / W;              // rays per lane
    static constexpr int kThreads = kWave * W;
    static constexpr int kStreamG = kStreamStep / kThreads;  // FULL: records per lane per step
    static constexpr int kBatch = 256;                    // survivors gathered per flush batch
    static constexpr int kShare = kBatch / W;             // raster walk: batch entries per wave
    static constexpr int kListCap = kBatch + kStreamStep;  // block id list: < kBatch + one step
};

template <int W>
struct CullShared {
    unsigned ids[CullShape<W>::kListCap];
    float4 st0[CullShape<W>::kBatch];  // gathered records: plane 0
    float4 st1[CullShape<W>::kBatch];  //                   plane 1
    float4 st2[CullShape<W>::kBatch];  //                   (cyC, vol, id, 0)
    float4 st3[CullShape<W>::kBatch];  //                   screen box
    unsigned hit[CullShape<W>::kBatch];  // raster walk: record may touch the tile (box + edge tests)
    int counts[2][W];
    Box wave_box[W];
    unsigned shared_fx;
    unsigned regular;
    // Raster walk: per-pixel lexicographic (t, id) keys of the tile's 32 x 64 rays.
    unsigned long long keys[kTileRows][kWave];
};

// (t, id) packed so that unsigned order is lexicographic order: t >= 0 here (vol > 0,
// det > 0), so its bit pattern orders like the value.
__device__ __forceinline__ unsigned long long HitKey(float t, int id) {
    return (static_cast<unsigned long long>(__float_as_uint(t)) << 32) | static_cast<unsigned>(id);
}

// Raster walk of one survivor over the whole tile (tiles whose rays all use the same sample
// offset: fx depends only on the column = lane, fy only on the row). The screen box picks
// the contiguous column range (lanes) and row range (of 32) it can touch; those pixels are
// tested exactly, lane-parallel, 64 pixels per round (rows packed when the column range is
// narrow), and each hit is merged into the pixel's key with an LDS atomic min. Same exact
// test and the same lexicographic result as ExactTestAnyOrder; any wave may walk any
// survivor, so a tile's survivors are shared evenly by its waves.
__device__ __forceinline__ void RasterSurvivor(unsigned long long (*keys)[kWave], const Record& q, float vol, int id,
                                               const float4& sb, bool use_sb, float fx_lane, float fy_lane,
                                               int lane) {
    unsigned long long cm = ~0ull;
    unsigned rm = 0xFFFFFFFFu;
    if (use_sb) {
        cm = __ballot(fx_lane >= sb.x && fx_lane <= sb.y);
        rm = static_cast<unsigned>(__ballot(fy_lane >= sb.z && fy_lane <= sb.w));  // lanes >= 32: NaN
        if (cm == 0ull || rm == 0u) {
            return;
        }
    }
    const int c0 = __builtin_ctzll(cm), c1 = 63 - __builtin_clzll(cm);
    const int r0 = __builtin_ctz(rm), r1 = 31 - __builtin_clz(rm);
    const int ncols = c1 - c0 + 1;
    const int lg = ncols <= 1 ? 0 : 32 - __builtin_clz(static_cast<unsigned>(ncols - 1));  // ceil(log2)
    const int col = c0 + (lane & ((1 << lg) - 1));
    const int step = kWave >> lg;
#pragma unroll 1
    for (int rr = r0; rr <= r1; rr += step) {
        const int row = rr + (lane >> lg);
        const float fx = __shfl(fx_lane, col);
        const float fy = __shfl(fy_lane, row & (kTileRows - 1));
        if (col <= c1 && row <= r1) {
            const float eA = fmaf(fy, q.cyA, fmaf(fx, q.cxA, q.c0A));
            const float eB = fmaf(fy, q.cyB, fmaf(fx, q.cxB, q.c0B));
            const float eC = fmaf(fy, q.cyC, fmaf(fx, q.cxC, q.c0C));
            const float det = (eA + eB) + eC;
            // all E >= 0 and det > 0 (NaN anywhere fails: det is then NaN)
            if (fminf(fminf(eA, eB), eC) >= 0.f && det > 0.f) {
                const float t = vol / det;
                if (t < __builtin_inff()) {
                    __hip_atomic_fetch_min(&keys[row][col], HitKey(t, id), __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP);
                }
            }
        }
    }
}

// Per-tile source of candidate records for the cull stream: every record of the scene
// (FULL), or the id list the bin kernel built for the tile's super-tile (LIST).
struct CullSource {
    const unsigned* list;  // LIST: ids (this block's chunk of the super-tile list)
    unsigned count;        // LIST: number of ids
    unsigned step0;        // FULL: first record step of this block's chunk
    unsigned steps;        // FULL: record steps of this block's chunk
};

// Streams the tile's candidates, keeps those whose quantized screen box overlaps the tile's
// (bq) in a block-wide LDS id list, and walks the survivors in flushes: gather their records
// into LDS, then either the raster walk (RASTER: survivors shared by the waves) or, per wave,
// the wave-box filter and ExactTestAnyOrder over every survivor (the wave's rays only).
template <int W, bool SHARED, bool RASTER, bool LIST>
__device__ __forceinline__ void CullWalk(const TraceParams& p, CullShared<W>& sh, Rays<CullShape<W>::kR>& s,
                                         const Box& bb, const Box& wb, float fx_lane, float fy_lane,
                                         CullSource src) {
    using S = CullShape<W>;
    constexpr int R = S::kR;
    constexpr int kThreads = S::kThreads;
    constexpr int kBatch = S::kBatch;
    constexpr int G = LIST ? kListG : S::kStreamG;
    constexpr int kStep = kThreads * G;
    static_assert(G <= 32, "pass bits of a step live in one 32-bit mask");
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    const float4* __restrict__ sbox = p.screen_boxes;
    const uint2* __restrict__ qbox = p.qboxes;
    const bool block_sb = ScreenBoxUsable(bb);
    const bool wave_sb = ScreenBoxUsable(wb);
    const QBox bq = Quantize(bb);
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const unsigned nsteps = LIST ? (src.count + kStep - 1) / kStep : src.steps;

    if constexpr (RASTER) {
        for (int i = tid; i < kTileRows * kWave; i += kThreads) {
            (&sh.keys[0][0])[i] = ~0ull;
        }  // visible to every wave after the first stream barrier
    }
#ifdef SRT_DIAG
    unsigned long long d_stream = 0, d_gather = 0, d_walk = 0, d_surv = 0, d_wsurv = 0, d_batches = 0;
    const unsigned long long d_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long d_mark = d_t0;
#endif
    // FULL: lane tid of step k reads records k * kStep + 2 * (l * kThreads + tid) + {0, 1}
    //       (one 16-B load per record pair); LIST: ids k * kStep + 4 * tid + {0..3} of the
    //       list (one 16-B load) and their 8-B boxes. The whole step is loaded one step ahead.
    constexpr int L = LIST ? 1 : G / 2;
    const uint4* __restrict__ qbox4 = reinterpret_cast<const uint4*>(qbox);
    uint4 nb[L];
    uint4 nid = make_uint4(0u, 0u, 0u, 0u);
    uint2 nq[LIST ? kListG : 1];
    auto fetch = [&](unsigned k) {
        if constexpr (LIST) {
            const unsigned i0 = k * kStep + 4 * tid;
            nid = i0 < src.count ? *reinterpret_cast<const uint4*>(src.list + i0) : make_uint4(0u, 0u, 0u, 0u);
            const unsigned v[4] = {nid.x, nid.y, nid.z, nid.w};
#pragma unroll
            for (int g = 0; g < kListG; ++g) {
                nq[g] = (i0 + g < src.count) ? qbox[v[g]] : make_uint2(0x80018001u, 0x80018001u);  // empty box
            }
        } else {
#pragma unroll
            for (int l = 0; l < L; ++l) {
                nb[l] = qbox4[(src.step0 + k) * (kStep / 2) + l * kThreads + tid];
            }
        }
    };
    if (nsteps > 0) {
        fetch(0);
    }
    int total = 0;  // ids in the block list (block-uniform)
    for (unsigned k = 0; k < nsteps; ++k) {
        uint4 cb[L];
        uint2 cq[LIST ? kListG : 1];
        const uint4 cid = nid;
#pragma unroll
        for (int l = 0; l < L; ++l) {
            cb[l] = nb[l];
        }
#pragma unroll
        for (int g = 0; g < (LIST ? kListG : 1); ++g) {
            cq[g] = nq[g];
        }
        if (k + 1 < nsteps) {
            fetch(k + 1);
        }
        auto record_id = [&](int g) -> unsigned {
            if constexpr (LIST) {
                return g == 0 ? cid.x : (g == 1 ? cid.y : (g == 2 ? cid.z : cid.w));
            } else {
                return (src.step0 + k) * kStep + 2 * ((g >> 1) * kThreads + tid) + (g & 1);
            }
        };
        unsigned bits = 0u;
        int wave_n = 0;
#pragma unroll
        for (int g = 0; g < G; ++g) {
            unsigned qx, qy;
            if constexpr (LIST) {
                qx = cq[g].x;
                qy = cq[g].y;
            } else {
                qx = (g & 1) ? cb[g >> 1].z : cb[g >> 1].x;
                qy = (g & 1) ? cb[g >> 1].w : cb[g >> 1].y;
            }
            // Disabled records carry empty boxes; unbounded ones span the int16 range. LIST
            // padding lanes carry an empty box too (and LIST implies a usable tile box).
            const bool pass = !block_sb || QBoxOverlaps(bq, qx, qy);
            bits |= pass ? (1u << g) : 0u;
            wave_n += __popcll(__ballot(pass));
        }
        const unsigned ph = k & 1u;
        if (lane == 0) {
            sh.counts[ph][wave] = wave_n;
        }
        __syncthreads();
        int off = total;
        int step_n = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int cw = sh.counts[ph][w];
            off += w < wave ? cw : 0;
            step_n += cw;
        }
        if (bits != 0u || step_n != 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const bool pass = (bits >> g) & 1u;
                const unsigned long long m = __ballot(pass);
                if (pass) {
                    sh.ids[off + __popcll(m & lt_mask)] = record_id(g);
                }
                off += __popcll(m);
            }
        }
        total += step_n;
        if (total < kBatch && k + 1 < nsteps) {  // block-uniform
            continue;
        }
        __syncthreads();  // every wave's ids are in the list
#ifdef SRT_DIAG
        {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            d_stream += now - d_mark;
            d_mark = now;
            d_surv += total;
        }
#endif
        // Flush: gather every listed record in batches of kBatch, then walk.
#pragma unroll 1
        for (int b0 = 0; b0 < total; b0 += kBatch) {
            const int e = b0 + tid;
            if (tid >= kBatch) {
                // not a gathering thread
            } else if (e < total) {
                const unsigned id = sh.ids[e];
                float4 p0, p1;
                float cyC, vol;
                LoadRecord(p.edges, id, p0, p1, cyC, vol);
                const float4 sb = sbox[id];
                sh.st0[tid] = p0;
                sh.st1[tid] = p1;
                sh.st2[tid] = make_float4(cyC, vol, __uint_as_float(id), 0.f);
                sh.st3[tid] = sb;
                if constexpr (RASTER) {
                    const Record r{p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, cyC};
                    sh.hit[tid] = ((!block_sb || ScreenBoxOverlaps(bb, sb)) && BoxMayHit(bb, r)) ? 1u : 0u;
                }
            } else if constexpr (RASTER) {
                sh.hit[tid] = 0u;
            }
            __syncthreads();
#ifdef SRT_DIAG
            {
                const unsigned long long now = __builtin_amdgcn_s_memtime();
                d_gather += now - d_mark;
                d_mark = now;
                ++d_batches;
            }
#endif
            const int nb_here = min(kBatch, total - b0);
            if constexpr (RASTER) {
                // This wave's share of the batch: entries wave * 64 .. wave * 64 + 63.
                const int c0 = wave * S::kShare;
                unsigned long long m = __ballot(lane < S::kShare && sh.hit[c0 + lane] != 0u);
#ifdef SRT_DIAG
                d_wsurv += __popcll(m);
#endif
                if (m != 0ull) {
                    // Software-pipelined: the next survivor's LDS reads are issued before the
                    // current one is walked, so their latency hides behind its work.
                    int bit = __builtin_ctzll(m);
                    float4 a = sh.st0[c0 + bit], b = sh.st1[c0 + bit], x = sh.st2[c0 + bit], sb = sh.st3[c0 + bit];
                    for (;;) {
                        m &= m - 1ull;
                        const bool more = m != 0ull;
                        const int nbit = more ? __builtin_ctzll(m) : bit;
                        const float4 an = sh.st0[c0 + nbit], bn = sh.st1[c0 + nbit], xn = sh.st2[c0 + nbit],
                                     sbn = sh.st3[c0 + nbit];
                        const Record r{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, x.x};
                        RasterSurvivor(sh.keys, r, x.y, __float_as_int(x.z), sb, block_sb, fx_lane, fy_lane, lane);
                        if (!more) {
                            break;
                        }
                        a = an;
                        b = bn;
                        x = xn;
                        sb = sbn;
                    }
                }
            } else {
#pragma unroll 1
                for (int c0 = 0; c0 < nb_here; c0 += kWave) {
                    const int i = c0 + lane;
                    bool pass = false;
                    if (i < nb_here) {
                        const float4 a = sh.st0[i], b = sh.st1[i], x = sh.st2[i];
                        const Record r{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, x.x};
                        pass = (!wave_sb || ScreenBoxOverlaps(wb, sh.st3[i])) && BoxMayHit(wb, r);
                    }
                    unsigned long long m = __ballot(pass);
#ifdef SRT_DIAG
                    d_wsurv += __popcll(m);
#endif
                    if (m != 0ull) {
                        int bit = __builtin_ctzll(m);
                        float4 a = sh.st0[c0 + bit], b = sh.st1[c0 + bit], x = sh.st2[c0 + bit];
                        for (;;) {
                            m &= m - 1ull;
                            const bool more = m != 0ull;
                            const int nbit = more ? __builtin_ctzll(m) : bit;
                            const float4 an = sh.st0[c0 + nbit], bn = sh.st1[c0 + nbit], xn = sh.st2[c0 + nbit];
                            const Record r{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, x.x};
                            ExactTestAnyOrder<R, SHARED>(s, r, x.y, __float_as_int(x.z));
                            if (!more) {
                                break;
                            }
                            a = an;
                            b = bn;
                            x = xn;
                        }
                    }
                }
            }
            __syncthreads();  // staging (and, after the last batch, the id list) reused next
#ifdef SRT_DIAG
            {
                const unsigned long long now = __builtin_amdgcn_s_memtime();
                d_walk += now - d_mark;
                d_mark = now;
            }
#endif
        }
        total = 0;
    }
    if (nsteps == 0) {
        __syncthreads();  // raster keys initialised by every wave before the read-back
    }
#ifdef SRT_DIAG
    const unsigned blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    if (tid == 0 && blk < kDiagBlocks) {
        unsigned long long* d = g_srt_diag[blk];
        d[0] = d_stream;
        d[1] = d_gather;
        d[2] = d_walk;
        d[3] = d_surv;
        d[4] = d_wsurv;
        d[5] = d_batches;
        d[6] = __builtin_amdgcn_s_memtime() - d_t0;
        d[7] = (RASTER ? 1 : 0) | (LIST ? 2 : 0) | 4;
    }
#endif
    if constexpr (RASTER) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const unsigned long long key = sh.keys[wave * R + r][lane];
            if (key != ~0ull) {
                s.bt[r] = __uint_as_float(static_cast<unsigned>(key >> 32));
                s.bi[r] = static_cast<int>(static_cast<unsigned>(key));
            }
        }
    }
}

// Super-tile = kSuperTiles tiles side by side (128 x 32 pixels): the unit of the bin lists.
constexpr int kSuperTiles = 2;
constexpr int kBinThreads = 256;
constexpr int kBinG = 8;          // records per lane per bin step (4 x 16-B loads)
constexpr int kBinStep = kBinThreads * kBinG;
constexpr int kBinMaxSlices = 32;  // bin blocks per super-tile row, striding over the record steps
constexpr int kBinRowSupers = 64;  // super-tiles per row handled per pass (LDS box cache)
constexpr unsigned kUnbinned = 0xFFFFFFFFu;
static_assert(kPadTriangles % kBinStep == 0, "bin steps must tile the records");

struct BinParams {
    const uint2* __restrict__ qboxes;
    const float2* __restrict__ offsets;
    uint4* __restrict__ super_q;    // per super-tile: (QBox.x, QBox.y, usable, 0)
    unsigned* __restrict__ lists;   // per super-tile: capacity ids
    unsigned* __restrict__ counts;  // per super-tile
    unsigned long long* __restrict__ tile_keys;  // reset to "no hit" here
    unsigned* __restrict__ tile_done;            // reset to 0 here
    unsigned capacity;
    unsigned n_pad;
    int supers_x;
    int width;
    int row_count;
    int row_begin;
    float wf;
    float hf;
};

// Level 0 of the cull: one block per super-tile computes its ray box from the sample offsets
// (GenerateRays' expressions, clamped edges included), stores it quantized for the bin
// kernel and resets the super-tile's list count (kUnbinned when the box lies outside the
// screen-box range: its tiles then stream every record).
__global__ __launch_bounds__(kBinThreads) void SuperBoxKernel(BinParams p) {
    constexpr int kWaves = kBinThreads / kWave;
    __shared__ Box boxes[kWaves];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const unsigned super = blockIdx.y * gridDim.x + blockIdx.x;
    const int x0 = blockIdx.x * kSuperTiles * kWave;
    const int y0 = blockIdx.y * kTileRows;
    Box box{__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()};
    for (int i = tid; i < kSuperTiles * kWave * kTileRows; i += kBinThreads) {
        const int xc = min(x0 + i % (kSuperTiles * kWave), p.width - 1);
        const int yc = min(y0 + i / (kSuperTiles * kWave), p.row_count - 1);
        const float2 o = p.offsets[static_cast<size_t>(yc) * p.width + xc];
        const float fx = (static_cast<float>(xc) + o.x) / p.wf;
        const float fy = (static_cast<float>(p.row_begin + yc) + o.y) / p.hf;
        box = Box{fminf(box.xlo, fx), fmaxf(box.xhi, fx), fminf(box.ylo, fy), fmaxf(box.yhi, fy)};
    }
    box = WaveReduceBox(box);
    if (lane == 0) {
        boxes[wave] = box;
    }
    __syncthreads();
    if (tid == 0) {
        box = boxes[0];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) {
            const Box o = boxes[w];
            box = Box{fminf(box.xlo, o.xlo), fmaxf(box.xhi, o.xhi), fminf(box.ylo, o.ylo), fmaxf(box.yhi, o.yhi)};
        }
        const bool usable = ScreenBoxUsable(box);
        const QBox q = Quantize(box);
        p.super_q[super] = make_uint4(q.x, q.y, usable ? 1u : 0u, 0u);
        p.counts[super] = usable ? 0u : kUnbinned;
    }
    // Split-tile state of the super-tile's pixels and tiles for this frame.
    const int tiles_x = (p.width + kWave - 1) / kWave;
    if (tid < kSuperTiles) {
        const int tx = blockIdx.x * kSuperTiles + tid;
        if (tx < tiles_x) {
            p.tile_done[blockIdx.y * tiles_x + tx] = 0u;
        }
    }
    for (int i = tid; i < kSuperTiles * kWave * kTileRows; i += kBinThreads) {
        const int xx = x0 + i % (kSuperTiles * kWave);
        const int yy = y0 + i / (kSuperTiles * kWave);
        if (xx < p.width && yy < p.row_count) {
            p.tile_keys[static_cast<size_t>(yy) * p.width + xx] = ~0ull;
        }
    }
}

// Level 1 of the cull (bin kernel): block (super-tile row, slice) streams the quantized
// screen boxes of its share of the records once and tests each against the row's box (the
// union of its super-tiles' boxes); each record that passes (a few percent) is then tested
// against every super-tile of the row at once, lane j taking super-tile j. Survivors are
// collected as (super-tile, id) pairs in wave-private LDS regions and flushed to the global
// lists with one atomic per super-tile per flush. Every record is still tested against
// every super-tile. A list that overflows its capacity makes the trace kernel stream every
// record for that super-tile instead.
constexpr int kBinWaves = kBinThreads / kWave;
constexpr int kBinWavePairs = 1024;                      // LDS pairs per wave region
constexpr int kBinPairCap = kBinWaves * kBinWavePairs;   // 4096
static_assert(kBinRowSupers <= kWave, "one super-tile per lane");
__global__ __launch_bounds__(kBinThreads) void BinKernel(BinParams p) {
    __shared__ unsigned pair_super[kBinPairCap];
    __shared__ unsigned pair_id[kBinPairCap];
    __shared__ unsigned wave_count[kBinWaves];
    __shared__ unsigned hist[kBinRowSupers];
    __shared__ unsigned gbase[kBinRowSupers];
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const unsigned row = blockIdx.x;
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    const unsigned nsteps = p.n_pad / kBinStep;
    const uint4* __restrict__ q4 = reinterpret_cast<const uint4*>(p.qboxes);
    constexpr int L = kBinG / 2;
    unsigned* my_super = pair_super + wave * kBinWavePairs;
    unsigned* my_id = pair_id + wave * kBinWavePairs;

    // Flush every wave's pairs: histogram per super-tile (LDS atomics give each pair its
    // rank), one global atomic per super-tile reserves list space, then scatter.
    auto flush = [&](int j0, int nj, unsigned mine) {
        if (lane == 0) {
            wave_count[wave] = mine;
        }
        if (tid < nj) {
            hist[tid] = 0u;
        }
        __syncthreads();
        unsigned rank[kBinPairCap / kBinThreads];
#pragma unroll
        for (int i = 0; i < kBinPairCap / kBinThreads; ++i) {
            const unsigned e = i * kBinThreads + tid;
            const bool valid = e % kBinWavePairs < wave_count[e / kBinWavePairs];
            rank[i] = valid ? atomicAdd(&hist[pair_super[e]], 1u) : 0u;
        }
        __syncthreads();
        if (tid < nj && hist[tid] != 0u) {
            gbase[tid] = atomicAdd(&p.counts[row * p.supers_x + j0 + tid], hist[tid]);
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < kBinPairCap / kBinThreads; ++i) {
            const unsigned e = i * kBinThreads + tid;
            if (e % kBinWavePairs < wave_count[e / kBinWavePairs]) {
                const unsigned j = pair_super[e];
                const unsigned at = gbase[j] + rank[i];
                if (at < p.capacity) {
                    p.lists[static_cast<size_t>(row * p.supers_x + j0 + j) * p.capacity + at] = pair_id[e];
                }
            }
        }
        __syncthreads();  // pair regions reused
    };

    for (int j0 = 0; j0 < p.supers_x; j0 += kBinRowSupers) {
        const int nj = min(kBinRowSupers, p.supers_x - j0);
        // Lane j < nj holds super-tile j's packed box (usable flag in .z).
        uint4 my_q = make_uint4(0x80008000u, 0x80008000u, 0u, 0u);
        if (lane < nj) {
            my_q = p.super_q[row * p.supers_x + j0 + lane];
        }
        const bool my_usable = my_q.z != 0u;
        const QBox my_box{my_q.x, my_q.y};
        // Row box: union of the usable super-tile boxes (in the packed (-lo, hi) form the
        // union is the per-half maximum).
        I16x2 ux = __builtin_bit_cast(I16x2, my_usable ? my_q.x : 0x80008000u);
        I16x2 uy = __builtin_bit_cast(I16x2, my_usable ? my_q.y : 0x80008000u);
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            ux = __builtin_elementwise_max(ux, __builtin_bit_cast(I16x2, __shfl_xor(__builtin_bit_cast(unsigned, ux), o)));
            uy = __builtin_elementwise_max(uy, __builtin_bit_cast(I16x2, __shfl_xor(__builtin_bit_cast(unsigned, uy), o)));
        }
        if (__ballot(my_usable) == 0ull) {
            continue;  // no usable super-tile in this part of the row
        }
        const QBox rq{__builtin_bit_cast(unsigned, ux), __builtin_bit_cast(unsigned, uy)};
        unsigned mine = 0;  // pairs in this wave's region (wave-uniform)
        for (unsigned k0 = blockIdx.y; k0 < nsteps; k0 += gridDim.y) {
            uint4 q[L];
#pragma unroll
            for (int l = 0; l < L; ++l) {
                q[l] = q4[k0 * (kBinStep / 2) + l * kBinThreads + tid];
            }
#pragma unroll
            for (int g = 0; g < kBinG; ++g) {
                const unsigned qx = (g & 1) ? q[g >> 1].z : q[g >> 1].x;
                const unsigned qy = (g & 1) ? q[g >> 1].w : q[g >> 1].y;
                unsigned long long m = __ballot(QBoxOverlaps(rq, qx, qy));
                // Each record of the row: every super-tile at once (lane j: super-tile j).
                while (m != 0ull) {
                    const int src = __builtin_ctzll(m);
                    m &= m - 1ull;
                    const unsigned rx = __builtin_amdgcn_readlane(qx, src);
                    const unsigned ry = __builtin_amdgcn_readlane(qy, src);
                    const bool hit = my_usable && QBoxOverlaps(my_box, rx, ry);
                    const unsigned long long hm = __ballot(hit);
                    if (hit) {
                        const unsigned at = mine + __popcll(hm & lt_mask);
                        my_super[at] = static_cast<unsigned>(lane);
                        my_id[at] = k0 * kBinStep + 2 * ((g >> 1) * kBinThreads + (wave * kWave + src)) + (g & 1);
                    }
                    mine += __popcll(hm);
                    if (mine + kWave > kBinWavePairs) {
                        // Region full: this wave's pairs go straight to the global lists.
                        unsigned gb = 0;
                        for (unsigned e = lane; e < mine; e += kWave) {
                            const unsigned j = my_super[e];
                            const unsigned at = atomicAdd(&p.counts[row * p.supers_x + j0 + j], 1u);
                            if (at < p.capacity) {
                                p.lists[static_cast<size_t>(row * p.supers_x + j0 + j) * p.capacity + at] = my_id[e];
                            }
                        }
                        (void)gb;
                        mine = 0;
                    }
                }
            }
            // Flush once some region is half full (block-uniform decision via LDS).
            if (lane == 0) {
                wave_count[wave] = mine;
            }
            __syncthreads();
            unsigned most = 0;
#pragma unroll
            for (int w = 0; w < kBinWaves; ++w) {
                most = max(most, wave_count[w]);
            }
            __syncthreads();
            if (most > kBinWavePairs / 2) {
                flush(j0, nj, mine);
                mine = 0;
            }
        }
        flush(j0, nj, mine);
    }
}

// How the blocks of one tile split its candidates: block z of chunks (blocks z >= chunks
// return at once). LIST: chunks of >= p.chunk_ids list ids (16-B aligned); FULL (a tile whose
// bin list overflowed, or no usable box): kMaxChunks slices of the record steps; without
// bins: one block.
constexpr unsigned kMaxChunks = 8;
struct CullPlan {
    CullSource src;
    unsigned chunks;
    bool list;
};
__device__ __forceinline__ CullPlan PlanTile(const TraceParams& p) {
    CullPlan plan{CullSource{nullptr, 0u, 0u, p.n_pad / kStreamStep}, 1u, false};
    if (p.bin_counts == nullptr) {
        return plan;
    }
    const unsigned super = blockIdx.y * ((gridDim.x + kSuperTiles - 1) / kSuperTiles) + blockIdx.x / kSuperTiles;
    const unsigned cnt = p.bin_counts[super];
    const unsigned z = blockIdx.z;
    if (cnt <= p.bin_capacity) {
        plan.list = true;
        plan.chunks = min(kMaxChunks, max(1u, (cnt + p.chunk_ids - 1) / p.chunk_ids));
        const unsigned per = ((cnt + plan.chunks - 1) / plan.chunks + 3u) & ~3u;
        const unsigned first = min(cnt, z * per);
        plan.src.list = p.bin_lists + static_cast<size_t>(super) * p.bin_capacity + first;
        plan.src.count = min(per, cnt - first);
    } else {
        const unsigned total = p.n_pad / kStreamStep;
        plan.chunks = min(kMaxChunks, total);
        const unsigned a = z * total / plan.chunks, b = (z + 1) * total / plan.chunks;
        plan.src.step0 = a;
        plan.src.steps = z < plan.chunks ? b - a : 0u;
    }
    return plan;
}

template <int W>
__global__ __launch_bounds__(kWave * W, (48 / W > 8 ? 8 : 48 / W)) void TraceCullKernel(TraceParams p) {
    using S = CullShape<W>;
    constexpr int R = S::kR;
    __shared__ CullShared<W> sh;
    if (p.bin_counts != nullptr) {
        const CullPlan early = PlanTile(p);
        if (blockIdx.z >= early.chunks) {
            return;  // this tile needs fewer blocks
        }
    }
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int x = blockIdx.x * kWave + lane;
    const int y0 = (blockIdx.y * W + wave) * R;
    Rays<R> s;
    Box lane_box;
    const bool same = GenerateRays<R>(p, x, y0, s, lane_box);
    const Box wb = WaveReduceBox(lane_box);
    // Raster walk eligibility: every ray of the tile has the tile's first sample offset
    // (bit pattern), so fx depends on the column only and fy on the row only.
    bool regular = true;
    float oy0;
    {
        const int x0 = min(static_cast<int>(blockIdx.x) * kWave, p.width - 1);
        const int yb = min(static_cast<int>(blockIdx.y) * kTileRows, p.row_count - 1);
        const float2 o0 = p.offsets[static_cast<size_t>(yb) * p.width + x0];
        oy0 = o0.y;
        const int xc = min(x, p.width - 1);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int yc = min(y0 + r, p.row_count - 1);
            const float2 o = p.offsets[static_cast<size_t>(yc) * p.width + xc];
            regular = regular && __float_as_uint(o.x) == __float_as_uint(o0.x) &&
                      __float_as_uint(o.y) == __float_as_uint(o0.y);
        }
    }
    if (tid == 0) {
        sh.shared_fx = 1u;
        sh.regular = 1u;
    }
    __syncthreads();
    if (lane == 0) {
        sh.wave_box[wave] = wb;
    }
    if (!__all(same) && lane == 0) {
        sh.shared_fx = 0u;
    }
    if (!__all(regular) && lane == 0) {
        sh.regular = 0u;
    }
    __syncthreads();
    Box bb = sh.wave_box[0];
#pragma unroll
    for (int w = 1; w < W; ++w) {
        const Box o = sh.wave_box[w];
        bb = Box{fminf(bb.xlo, o.xlo), fmaxf(bb.xhi, o.xhi), fminf(bb.ylo, o.ylo), fmaxf(bb.yhi, o.yhi)};
    }
    // Candidate source: the super-tile's bin list when it is complete, else every record;
    // split into `chunks` pieces taken by blocks z = 0 .. chunks-1 of this tile.
    const CullPlan plan = PlanTile(p);
    const CullSource& src = plan.src;
    const bool list = plan.list;
    // Raster walk: lane = column (fx), lanes 0..31 carry the tile's 32 rows' fy (the
    // GenerateRays expression; bit-identical since every ray has the same offset).
    const float fx_lane = s.fx[0];
    float fy_lane = __builtin_nanf("");
    if (lane < kTileRows) {
        const int yc = min(static_cast<int>(blockIdx.y) * kTileRows + lane, p.row_count - 1);
        fy_lane = (static_cast<float>(p.row_begin + yc) + oy0) / p.hf;
    }
    if (sh.regular != 0u && p.allow_raster != 0) {
        if (list) {
            CullWalk<W, true, true, true>(p, sh, s, bb, wb, fx_lane, fy_lane, src);
        } else {
            CullWalk<W, true, true, false>(p, sh, s, bb, wb, fx_lane, fy_lane, src);
        }
    } else if (sh.shared_fx != 0u) {
        if (list) {
            CullWalk<W, true, false, true>(p, sh, s, bb, wb, fx_lane, fy_lane, src);
        } else {
            CullWalk<W, true, false, false>(p, sh, s, bb, wb, fx_lane, fy_lane, src);
        }
    } else {
        if (list) {
            CullWalk<W, false, false, true>(p, sh, s, bb, wb, fx_lane, fy_lane, src);
        } else {
            CullWalk<W, false, false, false>(p, sh, s, bb, wb, fx_lane, fy_lane, src);
        }
    }
    if (plan.chunks > 1) {
        // Several blocks share this tile: merge this block's hits into the tile's global
        // keys (atomic min = the same lexicographic (t, id) rule), and the last block to
        // finish (agent-scope release/acquire around a per-tile counter) shades the tile.
        const int xc = min(x, p.width - 1);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int yc = min(y0 + r, p.row_count - 1);
            if (s.bi[r] >= 0) {
                atomicMin(&p.tile_keys[static_cast<size_t>(yc) * p.width + xc], HitKey(s.bt[r], s.bi[r]));
            }
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            const unsigned done = atomicAdd(&p.tile_done[blockIdx.y * gridDim.x + blockIdx.x], 1u);
            sh.shared_fx = done + 1u == plan.chunks ? 1u : 0u;  // reused as the "last block" flag
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        __syncthreads();
        if (sh.shared_fx == 0u) {
            return;
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int yc = min(y0 + r, p.row_count - 1);
            const unsigned long long key = __hip_atomic_load(&p.tile_keys[static_cast<size_t>(yc) * p.width + xc],
                                                             __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s.bt[r] = key == ~0ull ? __builtin_inff() : __uint_as_float(static_cast<unsigned>(key >> 32));
            s.bi[r] = key == ~0ull ? -1 : static_cast<int>(static_cast<unsigned>(key));
        }
    }
    ShadeAndStore<R>(p, x, y0, s);
}

// Waves per cull tile; env SRT_CULL_WAVES = 4, 8 or 16 (default 8), for measurement.
int CullWavesFromEnv() {
    const char* v = std::getenv("SRT_CULL_WAVES");
    if (v != nullptr && (std::strcmp(v, "4") == 0 || std::strcmp(v, "16") == 0)) {
        return std::atoi(v);
    }
    return 8;
}

}  // namespace

#ifdef SRT_DIAG
hipError_t DiagRead(void* host, std::size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_srt_diag), bytes < sizeof(g_srt_diag) ? bytes : sizeof(g_srt_diag));
}
#endif

hipError_t LaunchPrepare(const float* d_vertices, std::uint64_t n, const Frame& frame, float* d_edges,
                         hipStream_t stream) {
    PrepareParams p{};
    p.vertices = d_vertices;
    p.edges = reinterpret_cast<float4*>(d_edges);
    p.screen_boxes = reinterpret_cast<float4*>(d_edges) + PaddedTriangleCount(n) / kTileTriangles * kTileFloat4;
    p.qboxes = reinterpret_cast<uint2*>(p.screen_boxes + PaddedTriangleCount(n));
    p.n = static_cast<unsigned>(n);
    p.n_pad = static_cast<unsigned>(PaddedTriangleCount(n));
    for (int k = 0; k < 3; ++k) {
        p.origin[k] = frame.origin[k];
        p.base[k] = frame.base[k];
        p.du[k] = frame.du[k];
        p.dv[k] = frame.dv[k];
    }
    const unsigned blocks = (p.n_pad + 255) / 256;
    hipLaunchKernelGGL(PrepareKernel, dim3(blocks), dim3(256), 0, stream, p);
    return hipGetLastError();
}

std::size_t CullTiles(std::size_t width, std::size_t row_count) {
    return (width + kWave - 1) / kWave * ((row_count + kTileRows - 1) / kTileRows);
}

std::size_t CullSuperTiles(std::size_t width, std::size_t row_count) {
    const std::size_t gx = (width + kWave - 1) / kWave;
    const std::size_t gy = (row_count + kTileRows - 1) / kTileRows;
    return (gx + kSuperTiles - 1) / kSuperTiles * gy;
}

unsigned CullBinCapacity(std::uint64_t n, std::size_t supers) {
    const std::uint64_t n_pad = PaddedTriangleCount(n);
    std::uint64_t cap = supers == 0 ? n_pad : 64 * n_pad / supers;
    cap = cap < 4096 ? 4096 : cap;
    cap = cap > n_pad ? n_pad : cap;
    if (const char* v = std::getenv("SRT_CULL_BIN_CAP")) {  // tests: force list overflow
        const long forced = std::strtol(v, nullptr, 10);
        if (forced > 0) {
            cap = static_cast<std::uint64_t>(forced);
        }
    }
    return static_cast<unsigned>((cap + 3) / 4 * 4);
}

hipError_t LaunchTrace(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_albedo,
                       const Frame& frame, const float background[3], const BandArgs& band, int variant,
                       const CullBins* bins, hipStream_t stream) {
    if (band.row_count == 0 || band.width == 0) {
        return hipSuccess;
    }
    TraceParams p{};
    p.edges = reinterpret_cast<const float4*>(d_edges);
    p.screen_boxes = reinterpret_cast<const float4*>(d_edges) + PaddedTriangleCount(n) / kTileTriangles * kTileFloat4;
    p.qboxes = reinterpret_cast<const uint2*>(p.screen_boxes + PaddedTriangleCount(n));
    p.vertices = d_vertices;
    p.albedo = d_albedo;
    p.offsets = reinterpret_cast<const float2*>(band.offsets);
    p.out = reinterpret_cast<float4*>(band.rgba);
    p.n_pad = static_cast<unsigned>(PaddedTriangleCount(n));
    p.n_tiles = static_cast<unsigned>(n == 0 ? 1 : (n + kTileTriangles - 1) / kTileTriangles);
    p.width = static_cast<int>(band.width);
    p.row_count = static_cast<int>(band.row_count);
    p.row_begin = static_cast<int>(band.row_begin);
    {
        const char* r = std::getenv("SRT_CULL_RASTER");
        p.allow_raster = (r != nullptr && std::strcmp(r, "0") == 0) ? 0 : 1;
        const char* c = std::getenv("SRT_CULL_CHUNK");
        const long chunk = c != nullptr ? std::strtol(c, nullptr, 10) : 0;
        p.chunk_ids = chunk >= 64 ? static_cast<unsigned>(chunk) : 512u;
    }
    p.wf = static_cast<float>(band.width);
    p.hf = static_cast<float>(band.height);
    for (int k = 0; k < 3; ++k) {
        p.base[k] = frame.base[k];
        p.du[k] = frame.du[k];
        p.dv[k] = frame.dv[k];
        p.bg[k] = background[k];
    }
    const unsigned gx = static_cast<unsigned>((band.width + kWave - 1) / kWave);
    if (variant == kTraceScalar) {
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerLane - 1) / kRowsPerLane);
        hipLaunchKernelGGL(TraceScalarKernel, dim3(gx, gy), dim3(kWave), 0, stream, p);
    } else if (variant == kTraceCull) {
        const unsigned gy = static_cast<unsigned>((band.row_count + kTileRows - 1) / kTileRows);
        if (bins != nullptr) {
            const unsigned sx = (gx + kSuperTiles - 1) / kSuperTiles;
            if (static_cast<std::size_t>(sx) * gy > bins->supers) {
                return hipErrorInvalidValue;  // bins sized for another band shape
            }
            BinParams b{};
            b.qboxes = p.qboxes;
            b.offsets = p.offsets;
            b.super_q = reinterpret_cast<uint4*>(bins->super_q);
            b.lists = bins->lists;
            b.counts = bins->counts;
            b.tile_keys = reinterpret_cast<unsigned long long*>(bins->tile_keys);
            b.tile_done = bins->tile_done;
            b.capacity = bins->capacity;
            b.n_pad = p.n_pad;
            b.supers_x = static_cast<int>(sx);
            b.width = p.width;
            b.row_count = p.row_count;
            b.row_begin = p.row_begin;
            b.wf = p.wf;
            b.hf = p.hf;
            hipLaunchKernelGGL(SuperBoxKernel, dim3(sx, gy), dim3(kBinThreads), 0, stream, b);
            const unsigned slices = std::min<unsigned>(kBinMaxSlices, p.n_pad / kBinStep);
            hipLaunchKernelGGL(BinKernel, dim3(gy, slices), dim3(kBinThreads), 0, stream, b);
            p.bin_lists = bins->lists;
            p.bin_counts = bins->counts;
            p.bin_capacity = bins->capacity;
            p.tile_keys = b.tile_keys;
            p.tile_done = b.tile_done;
        }
        const unsigned gz = bins != nullptr ? kMaxChunks : 1u;
        switch (CullWavesFromEnv()) {
            case 4: hipLaunchKernelGGL(TraceCullKernel<4>, dim3(gx, gy, gz), dim3(kWave * 4), 0, stream, p); break;
            case 16: hipLaunchKernelGGL(TraceCullKernel<16>, dim3(gx, gy, gz), dim3(kWave * 16), 0, stream, p); break;
            default: hipLaunchKernelGGL(TraceCullKernel<8>, dim3(gx, gy, gz), dim3(kWave * 8), 0, stream, p); break;
        }
    } else {
        constexpr int kRowsPerBlock = kRowsPerLane * kLdsWaves;
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerBlock - 1) / kRowsPerBlock);
        hipLaunchKernelGGL(TraceLdsKernel, dim3(gx, gy), dim3(kWave * kLdsWaves), 0, stream, p);
    }
    return hipGetLastError();
}

}  // namespace srt
