// MI355X (gfx950) render kernels: edge-record preparation and the brute-force closest-hit
// trace. The reference has no render code; this file implements the
// north_star stages (a9)-(a12) of SURVEY.md section 8(a) from the canonical math in
// DESIGN.md. Built with -ffp-contract=off: every fused multiply-add below is an explicit
// fmaf, so CPU (oracle/srt_oracle.c) and GPU evaluate bit-identical float expressions.
#include "render.h"

#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <stdexcept>

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

// Cull record (the binned cull path's copy of one edge record, 64 B, stored at the record's
// rank in the scene's spatial order): a = (c0A, cxA, cyA, c0B), b = (cxB, cyB, c0C, cxC),
// x = (cyC, vol, id bits, 0), sb = screen box.
struct CullRecord {
    float4 a, b, x, sb;
};

// Per-tile facts the cull trace and the bin kernel share (TileInfoKernel), 32 B.
struct TileInfo {
    float4 box;         // (xlo, xhi, ylo, yhi) of the tile's ray positions (NaN positions drop out)
    float ox, oy;       // sample offset of the tile's first ray
    unsigned regular;   // every ray of the tile has offset (ox, oy), bit for bit
    unsigned usable;    // box within the screen-box range (else the tile streams every record)
};

struct TraceParams {
    const float4* __restrict__ edges;
    const float4* __restrict__ screen_boxes;
    const uint2* __restrict__ qboxes;
    const float* __restrict__ vertices;
    const float* __restrict__ albedo;
    const float4* __restrict__ normals;  // shading normals (PrepareRecord), by triangle id
    const float2* __restrict__ offsets;
    float4* __restrict__ out;
    unsigned n_pad;   // records in the edge buffer (multiple of kPadTriangles)
    unsigned n;       // records in the scene
    int tiles_x;         // cull tiles per tile row of the band
    unsigned tiles;      // cull tiles of the band
    unsigned n_tiles; // tiles holding at least one real record (>= 1)
    int width;
    int row_count;
    int row_begin;
    int allow_raster;  // cull variant: raster walk for uniform-offset tiles (env SRT_CULL_RASTER=0 disables)
    // Cull variant with bins (render.h CullBins); tile_info == null: no bins, every tile
    // computes its own ray box and streams every record.
    const TileInfo* __restrict__ tile_info;   // per tile: ray box, uniform offset (TileInfoKernel)
    const CullRecord* __restrict__ cull;      // cull records in spatial order (the lists hold positions)
    const unsigned* __restrict__ order;       // spatial-order position -> record id
    const unsigned* __restrict__ tile_order;  // block -> tile, most work first (TileOrderKernel)
    const unsigned* __restrict__ bin_lists;   // per tile: candidate ids (BinTrianglesKernel)
    const unsigned* __restrict__ bin_counts;  // per tile: list length; [tiles]: large-list length
    const unsigned* __restrict__ large_list;  // ids of records binned to every tile
    unsigned bin_capacity;
    unsigned exp;                                // diagnostic build: experiment bits (env SRT_EXP), 0 in the product
    float wf;
    float hf;
    float base[3];
    float du[3];
    float dv[3];
    float bg[3];
};

struct PrepareParams {
    const float* __restrict__ vertices;
    const unsigned* __restrict__ rank;  // record id -> position in the spatial order
    float4* __restrict__ edges;
    float4* __restrict__ screen_boxes;
    uint2* __restrict__ qboxes;
    CullRecord* __restrict__ cull;
    float4* __restrict__ normals;  // shading normal (e1 x e2, |e1 x e2|) per triangle id
    unsigned n;
    unsigned n_pad;
    float origin[3];
    float base[3];
    float du[3];
    float dv[3];
    unsigned exp;  // diagnostic build: experiment bits (env SRT_EXP), 0 in the product
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
__device__ __forceinline__ void PrepareRecord(const PrepareParams& p, unsigned i) {
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
    float4 sb = disabled ? make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff())
                         : make_float4(0.f, 0.f, 0.f, 0.f);
#ifdef SRT_DIAG
    if ((p.exp & 512u) == 0u && !disabled) {  // timing experiment: 512 skips the screen box
        sb = ScreenBox(c);
    }
#else
    if (!disabled) {
        sb = ScreenBox(c);
    }
#endif
    p.screen_boxes[i] = sb;
    // Stored as (hi, -lo) pairs so the cull test is one saturating packed add per axis.
    p.qboxes[i] = make_uint2(PackI16(QuantHi(sb.y), -QuantLo(sb.x)), PackI16(QuantHi(sb.w), -QuantLo(sb.z)));
    if (i < p.n) {
        // Shading normal, the exact expressions ShadeAndStore used to evaluate per hit.
        const float* v = p.vertices + 9ull * i;
        const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
        const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
        float nx, ny, nz;
        Cross3(e1x, e1y, e1z, e2x, e2y, e2z, nx, ny, nz);
        p.normals[i] = make_float4(nx, ny, nz, sqrtf(Dot3(nx, ny, nz, nx, ny, nz)));
        CullRecord r;
        r.a = make_float4(c[0], c[1], c[2], c[3]);
        r.b = make_float4(c[4], c[5], c[6], c[7]);
        r.x = make_float4(c[8], vol, __uint_as_float(i), 0.f);
        r.sb = sb;
#ifdef SRT_DIAG
        if (p.exp & 1024u) {  // timing experiment: coalesced record writes (wrong order)
            p.cull[i] = r;
            return;
        }
#endif
        p.cull[p.rank[i]] = r;
    }
}

__global__ __launch_bounds__(256) void PrepareKernel(PrepareParams p) {
    PrepareRecord(p, blockIdx.x * blockDim.x + threadIdx.x);
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
            const float4 nr = p.normals[id];  // (e1 x e2, |e1 x e2|) from the prepare kernel
            const float nd = Dot3(nr.x, nr.y, nr.z, dx, dy, dz);
            const float dd = Dot3(dx, dy, dz, dx, dy, dz);
            const float cosv = fminf(fabsf(nd) / (nr.w * sqrtf(dd)), 1.f);
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
constexpr int kTileRows = kCullTileRows;  // cull tile (bins): 64 columns x 32 rows
#ifndef SRT_BLOCK_ROWS
#define SRT_BLOCK_ROWS 16
#endif
constexpr int kBlockRows = SRT_BLOCK_ROWS;  // trace block: one part of a cull tile
constexpr int kParts = kTileRows / kBlockRows;
// Batch sizes of the cull walks (measured: these keep the trace block at 22 KB of LDS, up to
// 7 blocks per CU; the earlier 2048 / 512 / 256 took 35 KB, 4 blocks per CU, and 1.7 % longer).
#ifndef SRT_STREAM_STEP
#define SRT_STREAM_STEP 1024
#endif
#ifndef SRT_PACKET_BATCH
#define SRT_PACKET_BATCH 256
#endif
#ifndef SRT_PACKET_FLAT
// packet walk: 1 = a survivor's pixel range is cut row-major into packets of 64 pixels
// (ceil(cols*rows/64) packets); 0 = power-of-two-wide packets (2^lg columns x 64>>lg rows)
#define SRT_PACKET_FLAT 1
#endif
#ifndef SRT_PACKET_SPLIT
// packet walk (row-major packets): a survivor's range may be cut into two row bands, each with
// its own exact column range, when that takes fewer packets. Exact (GPU parity green) but
// measured slower: the six column searches in the gather phase cost more than the packets
// they save (trace 36.4 -> 43 us), so off by default.
#define SRT_PACKET_SPLIT 0
#endif
#ifndef SRT_PACKET_WORD
// packet walk (row-major packets, blocks of <= 16 rows): one packed word per packet
#define SRT_PACKET_WORD (SRT_PACKET_FLAT && SRT_BLOCK_ROWS <= 16)
#endif
#ifndef SRT_FAST_DIV
// packet walk (packed word path): t = vol / det by the IEEE sequence without its range
// scaling / fixup steps when vol and every candidate lane's det are in range (see
// EvalPacketFast). Exact (GPU parity green with it on) but measured slower: the per-packet
// ballot + uniform branch and the per-lane vol flag cost more than the 3 VALU they save
// (trace 36.5 -> 42.3 us), so off by default.
#define SRT_FAST_DIV 0
#endif
#ifndef SRT_PIN_LOADS
#define SRT_PIN_LOADS 1  // packet walk: pin loop-invariant lane values and keys (ISA scheduling)
#endif
#ifndef SRT_PACKET_ILP
#define SRT_PACKET_ILP 2  // packet walk: packets evaluated together per wave (independent chains)
#endif
#ifndef SRT_FLUSH_BATCH
#define SRT_FLUSH_BATCH 128
#endif
constexpr int kStreamStep = SRT_STREAM_STEP;  // FULL stream: records per block per step
constexpr int kListG = 4;          // LIST stream: ids per lane per step
constexpr int kPacketBatch = SRT_PACKET_BATCH;  // packet walk: survivors gathered per batch
static_assert(kPadTriangles % kStreamStep == 0, "a stream step must cover whole pad units");

// Block widths a build supports: at least one ray per lane and two streamed records per lane.
constexpr bool CullWavesOk(int w) { return kBlockRows / w >= 1 && kStreamStep / (kWave * w) >= 2; }

template <int W>
struct CullShape {
    static constexpr int kR = kBlockRows / W;             // rays per lane
    static constexpr int kThreads = kWave * W;
    static constexpr int kStreamG = kStreamStep / kThreads;  // FULL: records per lane per step
    static constexpr int kBatch = SRT_FLUSH_BATCH;        // survivors gathered per flush batch
    static constexpr int kShare = kBatch / W;             // raster walk: batch entries per wave
    static constexpr int kListStep = kThreads * kListG;     // LIST stream: ids per block per step
    static constexpr int kPBatch = kThreads > kPacketBatch ? kThreads : kPacketBatch;  // packet walk batch
    static constexpr int kListCap = kBatch + (kListStep > kStreamStep ? kListStep : kStreamStep);  // < kBatch + one step
};

template <int W>
struct CullShared {
    union {
        struct {  // stream walk (CullWalk)
            unsigned ids[CullShape<W>::kListCap];
            float4 st0[CullShape<W>::kBatch];  // gathered records: plane 0
            float4 st1[CullShape<W>::kBatch];  //                   plane 1
            float4 st2[CullShape<W>::kBatch];  //                   (cyC, vol, id, 0)
            float4 st3[CullShape<W>::kBatch];  //                   screen box
            unsigned hit[CullShape<W>::kBatch];  // raster walk: record may touch the tile (box + edge tests)
            int counts[2][W];
        } s;
        struct {  // packet walk (PacketWalk): one batch of compacted survivors
            float4 sv0[CullShape<W>::kPBatch];  // plane 0
            float4 sv1[CullShape<W>::kPBatch];  // plane 1
            float4 sv2[CullShape<W>::kPBatch];  // (cyC, vol, id, pixel range bits)
#if SRT_PACKET_SPLIT
            unsigned band2[CullShape<W>::kPBatch];  // second row band's range bits (split survivors)
#endif
            unsigned pre[CullShape<W>::kPBatch + 1];  // exclusive packet prefix, pre[S] = packets
            unsigned wave_n[CullShape<W>::kPBatch / kWave];   // survivors per (slice, wave)
            unsigned wave_pk[CullShape<W>::kPBatch / kWave];  // packets per (slice, wave)
            float fxs[kWave];                // fx of the tile's columns
            float fys[kBlockRows];           // fy of the block's rows
        } k;
    } u;
    Box wave_box[W];
    unsigned shared_fx;
    unsigned regular;
    // Raster walks: per-pixel lexicographic (t, id) keys of the tile's 32 x 64 rays.
    unsigned long long keys[kBlockRows][kWave];
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
        const float fy = __shfl(fy_lane, row & (kBlockRows - 1));
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
// (FULL), or (LIST) the tile's bin list followed by the large list (records binned to every
// tile), as one virtual list of which this block takes positions [begin, end).
struct CullSource {
    const unsigned* list;   // LIST: the tile's ids (virtual positions < count1)
    const unsigned* list2;  // LIST: large-list ids (virtual position v >= count1: list2[v - count1])
    unsigned count1;        // LIST: ids in the tile's list
    unsigned begin;         // LIST: this block's virtual positions [begin, end)
    unsigned end;
    unsigned step0;         // FULL: first record step of this block's chunk
    unsigned steps;         // FULL: record steps of this block's chunk
};

// Streams the tile's candidates, keeps those whose quantized screen box overlaps the tile's
// (bq) in a block-wide LDS id list, and walks the survivors in flushes: gather their records
// into LDS, then either the raster walk (RASTER: survivors shared by the waves) or, per wave,
// the wave-box filter and ExactTestAnyOrder over every survivor (the wave's rays only).
template <int W, bool SHARED, bool RASTER, bool LIST>
__device__ __forceinline__ void CullWalk(const TraceParams& p, CullShared<W>& sh, Rays<CullShape<W>::kR>& s,
                                         const Box& bb, const Box& wb, float fx_lane, float fy_lane,
                                         CullSource src, unsigned tile) {
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
    const unsigned nsteps = LIST ? (src.end - src.begin + kStep - 1) / kStep : src.steps;

    if constexpr (RASTER) {
        for (int i = tid; i < kBlockRows * kWave; i += kThreads) {
            (&sh.keys[0][0])[i] = ~0ull;
        }  // visible to every wave after the first stream barrier
    }
#ifdef SRT_DIAG
    unsigned long long d_stream = 0, d_gather = 0, d_walk = 0, d_surv = 0, d_wsurv = 0, d_batches = 0;
    const unsigned long long d_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long d_mark = d_t0;
#endif
    // FULL: lane tid of step k reads records k * kStep + 2 * (l * kThreads + tid) + {0, 1}
    //       (one 16-B load per record pair); LIST: virtual positions begin + k * kStep +
    //       g * kThreads + tid (coalesced 4-B id loads) and their 8-B boxes. The whole step is
    //       loaded one step ahead.
    constexpr int L = LIST ? 1 : G / 2;
    const uint4* __restrict__ qbox4 = reinterpret_cast<const uint4*>(qbox);
    uint4 nb[L];
    unsigned nid[LIST ? kListG : 1];
    uint2 nq[LIST ? kListG : 1];
    auto fetch = [&](unsigned k) {
        if constexpr (LIST) {
#pragma unroll
            for (int g = 0; g < kListG; ++g) {
                const unsigned v = src.begin + k * kStep + g * kThreads + tid;
                const bool in = v < src.end;
                nid[g] = in ? p.order[v < src.count1 ? src.list[v] : src.list2[v - src.count1]] : 0u;
            }
#pragma unroll
            for (int g = 0; g < kListG; ++g) {
                const unsigned v = src.begin + k * kStep + g * kThreads + tid;
                nq[g] = v < src.end ? qbox[nid[g]] : make_uint2(0x80018001u, 0x80018001u);  // empty box
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
        unsigned cid[LIST ? kListG : 1];
#pragma unroll
        for (int l = 0; l < L; ++l) {
            cb[l] = nb[l];
        }
#pragma unroll
        for (int g = 0; g < (LIST ? kListG : 1); ++g) {
            cq[g] = nq[g];
            cid[g] = nid[g];
        }
        if (k + 1 < nsteps) {
            fetch(k + 1);
        }
        auto record_id = [&](int g) -> unsigned {
            if constexpr (LIST) {
                return cid[g];
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
            sh.u.s.counts[ph][wave] = wave_n;
        }
        __syncthreads();
        int off = total;
        int step_n = 0;
#pragma unroll
        for (int w = 0; w < W; ++w) {
            const int cw = sh.u.s.counts[ph][w];
            off += w < wave ? cw : 0;
            step_n += cw;
        }
        if (bits != 0u || step_n != 0) {
#pragma unroll
            for (int g = 0; g < G; ++g) {
                const bool pass = (bits >> g) & 1u;
                const unsigned long long m = __ballot(pass);
                if (pass) {
                    sh.u.s.ids[off + __popcll(m & lt_mask)] = record_id(g);
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
                const unsigned id = sh.u.s.ids[e];
                float4 p0, p1;
                float cyC, vol;
                LoadRecord(p.edges, id, p0, p1, cyC, vol);
                const float4 sb = sbox[id];
                sh.u.s.st0[tid] = p0;
                sh.u.s.st1[tid] = p1;
                sh.u.s.st2[tid] = make_float4(cyC, vol, __uint_as_float(id), 0.f);
                sh.u.s.st3[tid] = sb;
                if constexpr (RASTER) {
                    const Record r{p0.x, p0.y, p0.z, p0.w, p1.x, p1.y, p1.z, p1.w, cyC};
                    sh.u.s.hit[tid] = ((!block_sb || ScreenBoxOverlaps(bb, sb)) && BoxMayHit(bb, r)) ? 1u : 0u;
                }
            } else if constexpr (RASTER) {
                sh.u.s.hit[tid] = 0u;
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
                unsigned long long m = __ballot(lane < S::kShare && sh.u.s.hit[c0 + lane] != 0u);
#ifdef SRT_DIAG
                d_wsurv += __popcll(m);
#endif
                if (m != 0ull) {
                    // Software-pipelined: the next survivor's LDS reads are issued before the
                    // current one is walked, so their latency hides behind its work.
                    int bit = __builtin_ctzll(m);
                    float4 a = sh.u.s.st0[c0 + bit], b = sh.u.s.st1[c0 + bit], x = sh.u.s.st2[c0 + bit], sb = sh.u.s.st3[c0 + bit];
                    for (;;) {
                        m &= m - 1ull;
                        const bool more = m != 0ull;
                        const int nbit = more ? __builtin_ctzll(m) : bit;
                        const float4 an = sh.u.s.st0[c0 + nbit], bn = sh.u.s.st1[c0 + nbit], xn = sh.u.s.st2[c0 + nbit],
                                     sbn = sh.u.s.st3[c0 + nbit];
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
                        const float4 a = sh.u.s.st0[i], b = sh.u.s.st1[i], x = sh.u.s.st2[i];
                        const Record r{a.x, a.y, a.z, a.w, b.x, b.y, b.z, b.w, x.x};
                        pass = (!wave_sb || ScreenBoxOverlaps(wb, sh.u.s.st3[i])) && BoxMayHit(wb, r);
                    }
                    unsigned long long m = __ballot(pass);
#ifdef SRT_DIAG
                    d_wsurv += __popcll(m);
#endif
                    if (m != 0ull) {
                        int bit = __builtin_ctzll(m);
                        float4 a = sh.u.s.st0[c0 + bit], b = sh.u.s.st1[c0 + bit], x = sh.u.s.st2[c0 + bit];
                        for (;;) {
                            m &= m - 1ull;
                            const bool more = m != 0ull;
                            const int nbit = more ? __builtin_ctzll(m) : bit;
                            const float4 an = sh.u.s.st0[c0 + nbit], bn = sh.u.s.st1[c0 + nbit], xn = sh.u.s.st2[c0 + nbit];
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
    const unsigned blk = blockIdx.z * gridDim.y * gridDim.x + tile;
    if (tid == 0 && blk < kDiagBlocks) {
        unsigned long long* d = g_srt_diag[blk];
        d[0] = d_stream;
        d[1] = d_gather;
        d[2] = d_walk;
        d[3] = d_surv;
        d[4] = d_wsurv;
        d[5] = d_batches;
        d[6] = __builtin_amdgcn_s_memtime() - d_t0;
        d[7] = (RASTER ? 1 : 0) | (LIST ? 2 : 0) | 4 |
               (p.bin_counts != nullptr ? (static_cast<unsigned long long>(p.bin_counts[tile]) << 16) |
                                              (static_cast<unsigned long long>(p.bin_counts[p.tiles]) << 40)
                                        : 0ull);
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

// ---------------------------------------------------------------------------------------
// Packet walk: binned tiles (LIST) whose rays all share one sample offset, so fx depends on
// the column only and fy on the row only, both monotone. Per batch of kPacketBatch list
// entries:
//   gather:  one thread per entry loads the record and its screen box, keeps it if it passes
//            the tile-box tests (ScreenBoxOverlaps, BoxMayHit), and finds the exact column
//            and row ranges of the tile whose ray positions lie inside the screen box (binary
//            searches in the tile's fx / fy tables). Pixels outside those ranges cannot pass
//            the exact test (screen-box guarantee), so skipping them is exact. The range is cut
//            into packets of 64 pixels (2^lg columns x 64 >> lg rows, 2^lg >= the width).
//   compact: survivors are compacted block-wide in any order, with an exclusive prefix of
//            their packet counts;
//   walk:    wave w takes the packets [w P / W, (w + 1) P / W) of the batch's P, two per
//            iteration (independent dependency chains for the scheduler): each lane tests
//            its pixel exactly and merges a hit into the pixel's key with an LDS atomic min.
// Same exact test and lexicographic (t, id) result as ExactTestAnyOrder.
// ---------------------------------------------------------------------------------------
// One packet (64 pixels of one survivor's range) evaluated without branches: the pixel's
// key and LDS address, and whether it is a hit (all E >= 0, det > 0, t finite; NaN anywhere
// fails). `bits` = the survivor's packed pixel range (wave-uniform), `j` = packet index.
struct PacketHit {
    unsigned long long key;
    unsigned addr;  // byte offset of the pixel's 8-B key in the tile's keys
    bool hit;
};

struct PacketPixel {
    unsigned colb, rowb;  // byte offsets of the pixel's column / row in the fx / fy tables
    bool in;
};

[[maybe_unused]] __device__ __forceinline__ PacketPixel PacketLane(unsigned bits, unsigned j, int lane) {
    const int c0 = bits & 63u, c1 = (bits >> 6) & 63u, r0 = (bits >> 12) & 31u, r1 = (bits >> 17) & 31u;
    const int lg = (bits >> 22) & 7u;
    const int col_u = c0 + (lane & ((1 << lg) - 1));
    const int row_u = r0 + static_cast<int>(j << (6 - lg)) + (lane >> lg);
    return PacketPixel{static_cast<unsigned>(min(col_u, c1)) * 4u, static_cast<unsigned>(min(row_u, r1)) * 4u,
                       static_cast<bool>((col_u <= c1) & (row_u <= r1))};
}

// Row-major packing: packet j of a survivor with range [c0, c0 + nc) x [r0, r0 + nr) covers
// range pixels p = 64 j + lane, p < nc * nr, at (c0 + p % nc, r0 + p / nc). p / nc is
// (p * m) >> 17 with m = ceil(2^17 / nc): exact, because p < 1088 and nc <= 64 keep
// p * (m - 2^17 / nc) / 2^17 < 1/nc (and p * m < 2^24 * 2^24 fits v_mul_u32_u24's low word,
// p * m < 2^32). Lanes past the range read padding-free table entries but are not `in`.
__device__ __forceinline__ unsigned PacketMagic(unsigned bits) {
    const unsigned nc = ((bits >> 6) & 63u) + 1u;
    return (131071u + nc) / nc;
}
__device__ __forceinline__ PacketPixel PacketLaneFlat(unsigned bits, unsigned j, unsigned m, int lane) {
    const unsigned c0 = bits & 63u, nc = ((bits >> 6) & 63u) + 1u, r0 = (bits >> 12) & 31u;
    const unsigned nr = ((bits >> 17) & 31u) + 1u;
    const unsigned pix = (j << 6) + static_cast<unsigned>(lane);
    const unsigned row_in = __umul24(pix, m) >> 17;  // pix < 2^11, m <= 2^17
    const unsigned col_in = pix - row_in * nc;
    return PacketPixel{(c0 + col_in) * 4u, (r0 + row_in) * 4u, pix < nc * nr};
}

// Row band split (SRT_PACKET_SPLIT). For rows [ra, rb] of the range, an edge function
// E = fma(fy, cy, fma(fx, cx, c0)) is monotone in fy (fma is monotone in each argument and the
// fy table is nondecreasing in the row), so its largest value over the band at column c is at
// fy* = fys[rb] (cy > 0) or fys[ra]; and at fixed fy* it is monotone in the column. The
// columns where E(fx_c, fy*) >= 0 are therefore a prefix or suffix of [lo, hi], found by
// binary search, and a column outside it fails that edge on every row of the band: dropping it
// is exact. NaN coefficients: E is NaN everywhere (no pixel passes), any cut is exact.
__device__ __forceinline__ void BandEdgeCut(const float* fxs, float fys_a, float fys_b, float cx, float cy, float c0,
                                            int c_lo, int c_hi, int& lo, int& hi) {
    // Branch-free lower bound over [c_lo, c_hi] (<= 64 columns, 7 fixed steps) of the first
    // column that does not "advance": for cx > 0 advance while E < 0 (the passing columns are
    // a suffix), for cx < 0 while E >= 0 (a prefix). cx == 0 (E constant in c) or NaN: one test.
    const float fy = cy > 0.f ? fys_b : fys_a;
    const bool inc = cx > 0.f;
    int pos = c_lo;
#pragma unroll
    for (int step = 64; step >= 1; step >>= 1) {
        const int c = pos + step - 1;
        const float e = fmaf(fy, cy, fmaf(fxs[min(c, c_hi)], cx, c0));
        pos += (c <= c_hi && ((e >= 0.f) != inc)) ? step : 0;
    }
    if (inc) {
        lo = pos;
        hi = c_hi;
    } else if (cx < 0.f) {
        lo = c_lo;
        hi = pos - 1;
    } else {
        const bool pass = fmaf(fy, cy, fmaf(fxs[c_lo], cx, c0)) >= 0.f;
        lo = c_lo;
        hi = pass ? c_hi : c_lo - 1;
    }
}

// Column range of rows [ra, rb] inside [c0, c1] (empty: c1 < c0 on return). The three edge
// cuts are independent searches over [c0, c1] (their LDS reads overlap), then intersected.
[[maybe_unused]] __device__ __forceinline__ void BandColumns(const float* fxs, const float* fys, const CullRecord& cr, int ra, int rb,
                                            int& c0, int& c1) {
    const float fa = fys[ra], fb = fys[rb];
    int l0, h0, l1, h1, l2, h2;
    BandEdgeCut(fxs, fa, fb, cr.a.y, cr.a.z, cr.a.x, c0, c1, l0, h0);
    BandEdgeCut(fxs, fa, fb, cr.b.x, cr.b.y, cr.a.w, c0, c1, l1, h1);
    BandEdgeCut(fxs, fa, fb, cr.b.w, cr.x.x, cr.b.z, c0, c1, l2, h2);
    c0 = max(max(l0, l1), l2);
    c1 = min(min(h0, h1), h2);
}

// One word per packet for the walk loop (one readlane instead of three): the range fields of
// PacketLaneFlat's `bits` narrowed to 4-bit rows, the survivor slot and the packet index.
// Needs rows < 16 (kBlockRows <= 16), slots < 256 and packets per survivor <= 16.
__device__ __forceinline__ unsigned PacketWord(unsigned bits, unsigned slot, unsigned j) {
    return (bits & 0xFFFu) | ((bits >> 12) & 15u) << 12 | ((bits >> 17) & 15u) << 16 | slot << 20 | j << 28;
}
__device__ __forceinline__ PacketPixel PacketLaneWord(unsigned w, unsigned m, int lane) {
    // In byte units (4 pix): (4 pix m) >> 19 == (pix m) >> 17, 4 pix m < 2^32.
    const unsigned c0 = w & 63u, nc = ((w >> 6) & 63u) + 1u, r0 = (w >> 12) & 15u, nr = ((w >> 16) & 15u) + 1u;
    const unsigned pix4 = (w >> 28 << 8) | (static_cast<unsigned>(lane) << 2);
    const unsigned row_in = __umul24(pix4, m) >> 19;
    return PacketPixel{pix4 + c0 * 4u - row_in * (nc * 4u), row_in * 4u + r0 * 4u, pix4 < nc * nr * 4u};
}

__device__ __forceinline__ PacketHit EvalPacket(const float4& a, const float4& b, const float4& x, float fx, float fy,
                                                const PacketPixel& px) {
    const float eA = fmaf(fy, a.z, fmaf(fx, a.y, a.x));
    const float eB = fmaf(fy, b.y, fmaf(fx, b.x, a.w));
    const float eC = fmaf(fy, x.x, fmaf(fx, b.w, b.z));
    const float det = (eA + eB) + eC;
    const float t = x.y / det;
    PacketHit h;
    h.hit = static_cast<bool>(px.in & (fminf(fminf(eA, eB), eC) >= 0.f) & (det > 0.f) & (t < __builtin_inff()));
    h.key = HitKey(t, __float_as_int(x.z));
    h.addr = px.rowb * (kWave * 2u) + px.colb * 2u;
    return h;
}

// EvalPacket with a cheaper exact division. The compiler's IEEE f32 division is
//   s = div_scale(det), n = div_scale(vol) [vcc], y = rcp(s), y = fma(fma(-s, y, 1), y, y),
//   q = n y, q = fma(fma(-s, q, n), y, q), q = div_fmas(fma(-s, q, n), y, q), div_fixup(q, det, vol)
// and div_scale leaves its operand unchanged (vcc = 0), div_fmas is then a plain fma, and
// div_fixup returns q, whenever vol and det are normal, nonzero, |exponent difference| < 96
// and the quotient is normal: true for vol in [2^-48, 2^48) and det in [2^-47, 2^47). Then
// the 8 instructions below give the same bits. vol is per survivor (vol_slow: outside its
// range), det per lane: if any lane that passes the edge tests has det outside its range (or
// vol_slow), the whole wave takes the IEEE division (a uniform branch) -- the fast path is an
// evaluation shortcut, never a change of result. On the fast path every passing lane has
// 0 < det and a finite t, so the hit is (edges pass) & (det in range).
[[maybe_unused]] __device__ __forceinline__ PacketHit EvalPacketFast(const float4& a, const float4& b, const float4& x, float fx,
                                                    float fy, const PacketPixel& px, bool vol_slow) {
    const float eA = fmaf(fy, a.z, fmaf(fx, a.y, a.x));
    const float eB = fmaf(fy, b.y, fmaf(fx, b.x, a.w));
    const float eC = fmaf(fy, x.x, fmaf(fx, b.w, b.z));
    const float det = (eA + eB) + eC;
    const bool e_ok = static_cast<bool>(px.in & (fminf(fminf(eA, eB), eC) >= 0.f));
    constexpr unsigned kLo = 0x28000000u, kHi = 0x57000000u;  // 2^-47, 2^47
    const bool det_ok = __float_as_uint(det) - kLo < kHi - kLo;
    PacketHit h;
    float t;
    if (vol_slow || __ballot(e_ok && !det_ok) != 0ull) {
        t = x.y / det;
        h.hit = static_cast<bool>(e_ok & (det > 0.f) & (t < __builtin_inff()));
    } else {
        const float y0 = __builtin_amdgcn_rcpf(det);
        const float y1 = fmaf(fmaf(-det, y0, 1.f), y0, y0);
        const float q0 = x.y * y1;
        const float q1 = fmaf(fmaf(-det, q0, x.y), y1, q0);
        t = fmaf(fmaf(-det, q1, x.y), y1, q1);
        h.hit = e_ok & det_ok;
    }
    h.key = HitKey(t, __float_as_int(x.z));
    h.addr = px.rowb * (kWave * 2u) + px.colb * 2u;
    return h;
}

// Range search in a nondecreasing table t[0..n): an index guess from a linear model, clamped
// to [0, n], then exact unit steps (a guess off by a few entries costs a few LDS reads).
__device__ __forceinline__ int GuessIndex(float v, float first, float scale, int n) {
    const float g = fminf(fmaxf((v - first) * scale, -1.f), static_cast<float>(n) + 1.f);  // NaN -> -1
    return g != g ? 0 : static_cast<int>(g);
}
// First i with t[i] >= v (n if none).
__device__ __forceinline__ int FirstAtLeast(const float* t, int n, float v, int g) {
    g = min(max(g, 0), n);
    while (g > 0 && t[g - 1] >= v) {
        --g;
    }
    while (g < n && t[g] < v) {
        ++g;
    }
    return g;
}
// Last i with t[i] <= v (-1 if none); g guesses the first i with t[i] > v.
__device__ __forceinline__ int LastAtMost(const float* t, int n, float v, int g) {
    g = min(max(g, 0), n);
    while (g > 0 && t[g - 1] > v) {
        --g;
    }
    while (g < n && t[g] <= v) {
        ++g;
    }
    return g - 1;
}

template <int W>
__device__ __forceinline__ void PacketWalk(const TraceParams& p, CullShared<W>& sh, Rays<CullShape<W>::kR>& s,
                                           const Box& bb, float fx_lane, float fy_lane, const CullSource& src, int tx,
                                           int row0) {
    using S = CullShape<W>;
    constexpr int R = S::kR;
    constexpr int kThreads = S::kThreads;
    constexpr int kBatchN = S::kPBatch;
    constexpr int kSlices = kBatchN / kThreads;  // batch entries per thread
    static_assert(kBatchN % kThreads == 0, "whole slices");
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    auto& k = sh.u.k;
#ifndef SRT_DIAG  // (the diag build records every block's counters)
    if (src.end == src.begin) {
        return;  // no candidates (block-uniform): every ray keeps its miss
    }
#endif
    const int nc = min(kWave, p.width - tx * kWave);
    const int nr = min(kBlockRows, p.row_count - row0);
    if (tid < kWave) {
        k.fxs[tid] = fx_lane;
    }
    if (tid < kBlockRows) {
        k.fys[tid] = fy_lane;
    }
    for (int i = tid; i < kBlockRows * kWave; i += kThreads) {
        (&sh.keys[0][0])[i] = ~0ull;
    }
    // Linear models of the (nondecreasing) column / row tables for the range guesses.
    const float fx_first = __shfl(fx_lane, 0), fx_last = __shfl(fx_lane, nc - 1);
    const float fy_first = __shfl(fy_lane, 0), fy_last = __shfl(fy_lane, nr - 1);
    const float fx_scale = nc > 1 && fx_last > fx_first ? static_cast<float>(nc - 1) / (fx_last - fx_first) : 0.f;
    const float fy_scale = nr > 1 && fy_last > fy_first ? static_cast<float>(nr - 1) / (fy_last - fy_first) : 0.f;
    __syncthreads();
    const unsigned total = src.end - src.begin;
#ifdef SRT_DIAG
    unsigned long long d_gather = 0, d_walk = 0, d_surv = 0, d_pk = 0, d_batches = 0;
    const unsigned long long d_t0 = __builtin_amdgcn_s_memtime();
    unsigned long long d_mark = d_t0;
#endif
    // Gather loads are software-pipelined one batch ahead: batch b+1's records are requested
    // before batch b's walk, so their latency hides behind it (heavy tiles take 2 batches).
    CullRecord nxt[kSlices];
    auto load_batch = [&](unsigned b0) {
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            const unsigned v = b0 + e * kThreads + tid;
            const unsigned vv = src.begin + (v < total ? v : 0u);
#ifdef SRT_DIAG
            if (p.exp & 256u) {  // timing experiment: coalesced loads (results wrong)
                nxt[e] = p.cull[(vv & 0xFFFFu) % p.n];
                continue;
            }
#endif
            nxt[e] = p.cull[vv < src.count1 ? src.list[vv] : src.list2[vv - src.count1]];
        }
    };
    if (total != 0u) {
        load_batch(0u);
    }
#pragma unroll 1
    for (unsigned b0 = 0; b0 < total; b0 += kBatchN) {
        // Gather: entries b0 + e * kThreads + tid of the block's virtual list.
        CullRecord cr[kSlices];
        bool pass[kSlices];
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            pass[e] = b0 + e * kThreads + tid < total;
            cr[e] = nxt[e];
        }
        unsigned bits[kSlices], npk[kSlices], band2[kSlices];
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            bits[e] = 0u;
            npk[e] = 0u;
            band2[e] = 0u;
            const float4 sb = cr[e].sb;
            const Record r{cr[e].a.x, cr[e].a.y, cr[e].a.z, cr[e].a.w, cr[e].b.x, cr[e].b.y, cr[e].b.z, cr[e].b.w,
                           cr[e].x.x};
            pass[e] = pass[e] && ScreenBoxOverlaps(bb, sb) && BoxMayHit(bb, r);
            if (pass[e]) {
                // Columns c with sb.xlo <= fx[c] <= sb.xhi (fx nondecreasing in c); rows likewise.
                // Interpolated guesses, then exact steps in the tables.
                const int c0 = FirstAtLeast(k.fxs, nc, sb.x, GuessIndex(sb.x, fx_first, fx_scale, nc));
                const int c1 = LastAtMost(k.fxs, nc, sb.y, GuessIndex(sb.y, fx_first, fx_scale, nc) + 1);
                const int r0 = FirstAtLeast(k.fys, nr, sb.z, GuessIndex(sb.z, fy_first, fy_scale, nr));
                const int r1 = LastAtMost(k.fys, nr, sb.w, GuessIndex(sb.w, fy_first, fy_scale, nr) + 1);
                pass[e] = c0 <= c1 && r0 <= r1;
                if (pass[e]) {
                    const int ncols = c1 - c0 + 1;
#if SRT_PACKET_FLAT
                    npk[e] = static_cast<unsigned>((ncols * (r1 - r0 + 1) + kWave - 1) / kWave);
                    bits[e] = static_cast<unsigned>(c0) | static_cast<unsigned>(ncols - 1) << 6 |
                              static_cast<unsigned>(r0) << 12 | static_cast<unsigned>(r1 - r0) << 17;
#if SRT_PACKET_SPLIT
                    if (npk[e] > 1u) {  // a one-packet range cannot get cheaper
                        const int rm = r0 + ((r1 - r0 + 1) >> 1);  // bands [r0, rm - 1], [rm, r1]
                        int a0 = c0, a1 = c1, b0 = c0, b1 = c1;
                        BandColumns(k.fxs, k.fys, cr[e], r0, rm - 1, a0, a1);
                        BandColumns(k.fxs, k.fys, cr[e], rm, r1, b0, b1);
                        const unsigned na = a0 <= a1 ? static_cast<unsigned>(((a1 - a0 + 1) * (rm - r0) + kWave - 1) / kWave) : 0u;
                        const unsigned nb = b0 <= b1 ? static_cast<unsigned>(((b1 - b0 + 1) * (r1 - rm + 1) + kWave - 1) / kWave) : 0u;
                        const unsigned bits_a = static_cast<unsigned>(a0) | static_cast<unsigned>(a1 - a0) << 6 |
                                                static_cast<unsigned>(r0) << 12 | static_cast<unsigned>(rm - 1 - r0) << 17;
                        const unsigned bits_b = static_cast<unsigned>(b0) | static_cast<unsigned>(b1 - b0) << 6 |
                                                static_cast<unsigned>(rm) << 12 | static_cast<unsigned>(r1 - rm) << 17;
                        if (na + nb < npk[e]) {
                            npk[e] = na + nb;
                            if (na == 0u) {
                                bits[e] = bits_b;
                            } else if (nb == 0u) {
                                bits[e] = bits_a;
                            } else {
                                bits[e] = bits_a | 1u << 22;
                                band2[e] = bits_b;
                            }
                            pass[e] = npk[e] != 0u;
                        }
                    }
#endif
#else
                    const int lg = ncols <= 1 ? 0 : 32 - __builtin_clz(static_cast<unsigned>(ncols - 1));
                    const int rpp = kWave >> lg;
                    npk[e] = static_cast<unsigned>((r1 - r0 + rpp) / rpp);
                    bits[e] = static_cast<unsigned>(c0) | static_cast<unsigned>(c1) << 6 |
                              static_cast<unsigned>(r0) << 12 | static_cast<unsigned>(r1) << 17 |
                              static_cast<unsigned>(lg) << 22;
#endif
                }
            }
        }
        // Compact the survivors block-wide ((slice, wave, lane) order); exclusive packet
        // prefix in compacted order.
        unsigned wpos[kSlices], incl[kSlices];
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            const unsigned long long m = __ballot(pass[e]);
            wpos[e] = __popcll(m & lt_mask);
            incl[e] = npk[e];
#pragma unroll
            for (int o = 1; o < kWave; o <<= 1) {
                const unsigned t = __shfl_up(incl[e], o);
                if (lane >= o) {
                    incl[e] += t;
                }
            }
            if (lane == kWave - 1) {
                k.wave_n[e * W + wave] = __popcll(m);
                k.wave_pk[e * W + wave] = incl[e];
            }
        }
        __syncthreads();
        // Bases of (slice e, this wave): the virtual waves (e', w') before it, in order.
        unsigned n_surv = 0, n_pk = 0;
        unsigned sbase[kSlices], pbase[kSlices];
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            sbase[e] = 0u;
            pbase[e] = 0u;
        }
#pragma unroll
        for (int vw = 0; vw < kSlices * W; ++vw) {
            const unsigned wn = k.wave_n[vw], wp = k.wave_pk[vw];
#pragma unroll
            for (int e = 0; e < kSlices; ++e) {
                const bool before = vw < e * W + wave;
                sbase[e] += before ? wn : 0u;
                pbase[e] += before ? wp : 0u;
            }
            n_surv += wn;
            n_pk += wp;
        }
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            if (pass[e]) {
                const unsigned slot = sbase[e] + wpos[e];
                k.sv0[slot] = cr[e].a;
                k.sv1[slot] = cr[e].b;
                k.sv2[slot] = make_float4(cr[e].x.x, cr[e].x.y, cr[e].x.z, __uint_as_float(bits[e]));
#if SRT_PACKET_SPLIT
                k.band2[slot] = band2[e];
#endif
                k.pre[slot] = pbase[e] + incl[e] - npk[e];
            }
        }
        if (tid == 0) {
            k.pre[n_surv] = n_pk;
        }
        __syncthreads();
#ifdef SRT_DIAG
        {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            d_gather += now - d_mark;
            d_mark = now;
            d_surv += n_surv;
            d_pk += n_pk;
            ++d_batches;
        }
#endif
        if (b0 + kBatchN < total) {
            load_batch(b0 + kBatchN);
        }
        // Walk this wave's packets [q_begin, q_end), 64 at a time: lane l finds packet q0 + l's
        // survivor (binary search in pre) and fetches its range bits, then the wave takes the
        // packets kPacketIlp at a time (independent chains: all LDS reads issued together; a
        // tail repeats the last packet, harmless under an atomic min) and applies the hits.
        constexpr int kPacketIlp = SRT_PACKET_ILP;
        unsigned q_begin = wave * n_pk / W, q_end = (wave + 1) * n_pk / W;
#ifdef SRT_DIAG
        if (p.exp & 64u) {
            q_end = q_begin;
        }
#endif
        unsigned long long* keys = &sh.keys[0][0];
#pragma unroll 1
        for (unsigned q0 = q_begin; q0 < q_end; q0 += kWave) {
            const unsigned mine = min(q0 + static_cast<unsigned>(lane), q_end - 1u);
            int lo = 0, hi = static_cast<int>(n_surv) - 1;  // last survivor with pre <= mine
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (k.pre[mid] <= mine) {
                    lo = mid;
                } else {
                    hi = mid - 1;
                }
            }
            const unsigned my_s = static_cast<unsigned>(lo);
            unsigned my_j = mine - k.pre[lo];
            unsigned my_bits = __float_as_uint(k.sv2[lo].w);
#if SRT_PACKET_FLAT && SRT_PACKET_SPLIT
            if (my_bits & (1u << 22)) {  // two row bands: the first band's packets come first
                const unsigned na = ((((my_bits >> 6) & 63u) + 1u) * (((my_bits >> 17) & 31u) + 1u) + kWave - 1) / kWave;
                if (my_j >= na) {
                    my_bits = k.band2[lo];
                    my_j -= na;
                }
            }
#endif
            const unsigned n = min(static_cast<unsigned>(kWave), q_end - q0);
#if SRT_PACKET_FLAT
            unsigned my_m = PacketMagic(my_bits);  // < 2^18; bit 31: vol outside the fast-division range
#if SRT_FAST_DIV
            {
                const unsigned vb = __float_as_uint(k.sv2[my_s].y);
                my_m |= vb - 0x27800000u < 0x57800000u - 0x27800000u ? 0u : 0x80000000u;  // [2^-48, 2^48)
            }
#endif
#endif
#if SRT_PACKET_WORD
            constexpr bool kWord = kBlockRows <= 16 && S::kPBatch <= 256;  // field widths
            const unsigned my_w = kWord ? PacketWord(my_bits, my_s, my_j) : 0u;
            if constexpr (kWord) {
                asm volatile("" ::"v"(my_w));
            }
#endif
#if SRT_PIN_LOADS
            // Resolve the per-lane packet table before the loop, so the loop header does not
            // wait for the previous iteration's LDS atomics (conservative waitcnt merge).
            asm volatile("" ::"v"(my_s), "v"(my_bits), "v"(my_j));
#if SRT_PACKET_FLAT
            asm volatile("" ::"v"(my_m));
#endif
#endif
#pragma unroll 1
            for (unsigned i = 0; i < n; i += kPacketIlp) {
                unsigned ps[kPacketIlp];
                PacketPixel px[kPacketIlp];
                float4 ra[kPacketIlp], rb[kPacketIlp], rx[kPacketIlp];
                float fx[kPacketIlp], fy[kPacketIlp];
                bool vol_slow[kPacketIlp];
#pragma unroll
                for (int u = 0; u < kPacketIlp; ++u) {
                    const unsigned li = min(i + u, n - 1u);
                    vol_slow[u] = true;
#if SRT_PACKET_WORD
                    if constexpr (kWord) {
                        const unsigned w = __builtin_amdgcn_readlane(my_w, li);
                        const unsigned mm = __builtin_amdgcn_readlane(my_m, li);
                        ps[u] = (w >> 20) & 255u;
                        vol_slow[u] = (mm >> 31) != 0u;
                        px[u] = PacketLaneWord(w, mm, lane);
                    } else {
                        ps[u] = __builtin_amdgcn_readlane(my_s, li);
                        px[u] = PacketLaneFlat(__builtin_amdgcn_readlane(my_bits, li),
                                               __builtin_amdgcn_readlane(my_j, li), __builtin_amdgcn_readlane(my_m, li),
                                               lane);
                    }
#elif SRT_PACKET_FLAT
                    ps[u] = __builtin_amdgcn_readlane(my_s, li);
                    px[u] = PacketLaneFlat(__builtin_amdgcn_readlane(my_bits, li), __builtin_amdgcn_readlane(my_j, li),
                                           __builtin_amdgcn_readlane(my_m, li), lane);
#else
                    ps[u] = __builtin_amdgcn_readlane(my_s, li);
                    px[u] = PacketLane(__builtin_amdgcn_readlane(my_bits, li), __builtin_amdgcn_readlane(my_j, li), lane);
#endif
                }
#pragma unroll
                for (int u = 0; u < kPacketIlp; ++u) {
                    ra[u] = k.sv0[ps[u]];
                    rb[u] = k.sv1[ps[u]];
                    rx[u] = k.sv2[ps[u]];
                    fx[u] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(k.fxs) + px[u].colb);
                    fy[u] = *reinterpret_cast<const float*>(reinterpret_cast<const char*>(k.fys) + px[u].rowb);
                }
                PacketHit h[kPacketIlp];
#pragma unroll
                for (int u = 0; u < kPacketIlp; ++u) {
#if SRT_FAST_DIV && SRT_PACKET_FLAT
                    h[u] = EvalPacketFast(ra[u], rb[u], rx[u], fx[u], fy[u], px[u], vol_slow[u]);
#else
                    (void)vol_slow[u];
                    h[u] = EvalPacket(ra[u], rb[u], rx[u], fx[u], fy[u], px[u]);
#endif
                }
#if SRT_PIN_LOADS
                // Keys built before the hit branches: the record id is loaded with the rest of
                // the record instead of by a separate LDS read (and full wait) inside the branch.
#pragma unroll
                for (int u = 0; u < kPacketIlp; ++u) {
                    asm volatile("" ::"v"(h[u].key));
                }
#endif
#pragma unroll
                for (int u = 0; u < kPacketIlp; ++u) {
#ifdef SRT_DIAG
                    if (p.exp & 32u) {
                        continue;
                    }
#endif
                    if (h[u].hit) {
                        __hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(
                                                   reinterpret_cast<char*>(keys) + h[u].addr),
                                               h[u].key, __ATOMIC_RELAXED,
                                               __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
        __syncthreads();  // batch storage reused; after the last batch: keys complete
#ifdef SRT_DIAG
        {
            const unsigned long long now = __builtin_amdgcn_s_memtime();
            d_walk += now - d_mark;
            d_mark = now;
        }
#endif
    }
#ifdef SRT_DIAG
    const unsigned blk = blockIdx.y * gridDim.x + blockIdx.x;
    if (tid == 0 && blk < kDiagBlocks) {
        unsigned long long* d = g_srt_diag[blk];
        d[0] = 0;
        d[1] = d_gather;
        d[2] = d_walk;
        d[3] = d_surv;
        d[4] = d_pk;
        d[5] = d_batches;
        d[6] = __builtin_amdgcn_s_memtime() - d_t0;
        d[7] = 1 | 2 | 4 | 8 | (static_cast<unsigned long long>(src.count1) << 16) |
               (static_cast<unsigned long long>(src.end - src.count1) << 40);
    }
#endif
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const unsigned long long key = sh.keys[wave * R + r][lane];
        if (key != ~0ull) {
            s.bt[r] = __uint_as_float(static_cast<unsigned>(key >> 32));
            s.bi[r] = static_cast<int>(static_cast<unsigned>(key));
        }
    }
}

// ---------------------------------------------------------------------------------------
// Cull bins: the first cull level, built per band before the trace. A tile is 64 x 32 rays
// (one trace block).
//   TileInfoKernel:     one block per tile reads the tile's sample offsets once: the ray
//                       box, "regular" (every offset equal to the first, bit for bit) and the
//                       first offset; it clears the tile's bin count.
//   BinTrianglesKernel: every block first reduces the tile boxes to per tile-column and per
//                       tile-row bounds, made monotone (suffix minimum of lo, prefix maximum
//                       of hi). Then one thread per record: binary searches in them give
//                       the contiguous range of tile columns and rows whose boxes can overlap
//                       the record's screen box; every tile of the range whose own box passes
//                       the screen-box overlap and the edge-function corner test (BoxMayHit)
//                       gets the id appended to its list. A record whose range spans more than
//                       kLargeTiles tiles (big, or an unbounded screen box) goes to the large
//                       list, which every binned tile walks after its own list.
// Both steps drop only (record, tile) pairs that provably fail the exact test for every ray
// of the tile, so the frame stays bit-identical to brute force. A tile whose box is outside
// the screen-box range, or whose list overflowed, streams every record instead.
// ---------------------------------------------------------------------------------------
constexpr int kBinThreads = 256;
constexpr int kLargeTiles = 16;  // records spanning more tiles go to the large list
static_assert(kTileRows == kCullTileRows && kWave == kCullTileCols, "render.h tile shape");

struct BinParams {
    const float2* __restrict__ offsets;
    const CullRecord* __restrict__ cull;  // cull records in spatial order
    TileInfo* __restrict__ tile_info;
    unsigned* __restrict__ counts;      // tiles + 1 (the last one: large list)
    unsigned* __restrict__ lists;       // tiles x capacity
    unsigned* __restrict__ large_list;  // n_pad
    unsigned* __restrict__ tile_order;  // tiles: trace block -> tile (TileOrderKernel)
    unsigned* __restrict__ sync;        // [0] bin blocks done (self-resetting)
    float2* __restrict__ bounds;        // tiles_x + tiles_y monotone tile column / row bounds (TileBoundsKernel)
    unsigned order_in_bin;              // the bin kernel's last block computes the tile order
    unsigned capacity;
    unsigned n;
    unsigned exp;  // diagnostic build: experiment bits (env SRT_EXP), 0 in the product
    int tiles_x;
    int tiles_y;
    int width;
    int row_count;
    int row_begin;
    float wf;
    float hf;
};

// Order-preserving map float -> unsigned, for LDS atomic min / max (no NaNs reach it).
__device__ __forceinline__ unsigned OrderedBits(float v) {
    const unsigned b = __float_as_uint(v);
    return (b & 0x80000000u) ? ~b : (b | 0x80000000u);
}
__device__ __forceinline__ float FromOrderedBits(unsigned k) {
    return __uint_as_float((k & 0x80000000u) ? (k & 0x7FFFFFFFu) : ~k);
}

// In-place inclusive scan (max, or min) of a[0..n) by one wave; `reverse` scans from the end.
template <bool MAX>
__device__ void WaveScanOrdered(unsigned* a, int n, bool reverse, int lane) {
    const unsigned ident = MAX ? OrderedBits(-__builtin_inff()) : OrderedBits(__builtin_inff());
    unsigned carry = ident;
    for (int c0 = 0; c0 < n; c0 += kWave) {
        const int i = c0 + lane;
        const int j = reverse ? n - 1 - i : i;
        unsigned v = i < n ? a[j] : ident;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const unsigned u = __shfl_up(v, o);
            if (lane >= o) {
                v = MAX ? max(v, u) : min(v, u);
            }
        }
        v = MAX ? max(v, carry) : min(v, carry);
        if (i < n) {
            a[j] = v;
        }
        carry = __shfl(v, kWave - 1);
    }
}

// One block per tile (bx, by).
__device__ __forceinline__ void TileInfoBlock(const BinParams& p, int bx, int by) {
    constexpr int kWaves = kBinThreads / kWave;
    constexpr int kPer = kWave * kTileRows / kBinThreads;  // offsets per thread (8)
    __shared__ Box boxes[kWaves];
    __shared__ unsigned irregular;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const int x0 = bx * kWave;
    const int y0 = by * kTileRows;
    if (tid == 0) {
        irregular = 0u;
    }
    // All loads first (clamped addresses: duplicates of real pixels), then the box. Same
    // expressions as GenerateRays; NaN positions drop out of the box (fminf / fmaxf).
    const float2 o0 = p.offsets[static_cast<size_t>(y0) * p.width + x0];
    const int xx = min(x0 + lane, p.width - 1);
    float2 o[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int yy = min(y0 + wave + k * kWaves, p.row_count - 1);
        o[k] = p.offsets[static_cast<size_t>(yy) * p.width + xx];
    }
    Box box{__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()};
    bool regular = true;
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const int yy = min(y0 + wave + k * kWaves, p.row_count - 1);
        const float fx = (static_cast<float>(xx) + o[k].x) / p.wf;
        const float fy = (static_cast<float>(p.row_begin + yy) + o[k].y) / p.hf;
        box = Box{fminf(box.xlo, fx), fmaxf(box.xhi, fx), fminf(box.ylo, fy), fmaxf(box.yhi, fy)};
        regular = regular && __float_as_uint(o[k].x) == __float_as_uint(o0.x) &&
                  __float_as_uint(o[k].y) == __float_as_uint(o0.y);
    }
    box = WaveReduceBox(box);
    const bool wave_regular = __all(regular);
    __syncthreads();  // `irregular` initialised
    if (lane == 0) {
        boxes[wave] = box;
        if (!wave_regular) {
            irregular = 1u;
        }
    }
    __syncthreads();
    if (tid == 0) {
        box = boxes[0];
#pragma unroll
        for (int w = 1; w < kWaves; ++w) {
            const Box b = boxes[w];
            box = Box{fminf(box.xlo, b.xlo), fmaxf(box.xhi, b.xhi), fminf(box.ylo, b.ylo), fmaxf(box.yhi, b.yhi)};
        }
        TileInfo ti;
        ti.box = make_float4(box.xlo, box.xhi, box.ylo, box.yhi);
        ti.ox = o0.x;
        ti.oy = o0.y;
        ti.regular = irregular == 0u ? 1u : 0u;
        ti.usable = ScreenBoxUsable(box) ? 1u : 0u;
        const unsigned tile = by * p.tiles_x + bx;
        p.tile_info[tile] = ti;
        p.counts[tile] = 0u;  // the bin kernel runs after this one (stream order)
        if (tile == 0) {
            p.counts[p.tiles_x * p.tiles_y] = 0u;  // large list
        }
    }
}

__global__ __launch_bounds__(kBinThreads) void TileInfoKernel(BinParams p) {
    TileInfoBlock(p, blockIdx.x, blockIdx.y);
}

// Prepare (one thread per record) and tile info (one block per tile) in one launch: block
// b < prep_blocks prepares records, the others are tile blocks. The two are independent
// (records vs sample offsets), so the latency-bound prepare blocks overlap the
// bandwidth-bound tile blocks.
struct PrepareInfoParams {
    PrepareParams prep;
    BinParams bin;
    unsigned prep_blocks;
};
__global__ __launch_bounds__(kBinThreads) void PrepareInfoKernel(PrepareInfoParams p) {
    static_assert(kBinThreads == 256, "prepare blocks are 256 threads");
    const unsigned b = blockIdx.x;
    if (b < p.prep_blocks) {
        PrepareRecord(p.prep, b * kBinThreads + threadIdx.x);
        return;
    }
    const unsigned t = b - p.prep_blocks;
    TileInfoBlock(p.bin, static_cast<int>(t % static_cast<unsigned>(p.bin.tiles_x)),
                  static_cast<int>(t / static_cast<unsigned>(p.bin.tiles_x)));
}

// First index i of the nondecreasing hi'[0..n) with hi'[i] >= v (n if none).
__device__ __forceinline__ int FirstHiAtLeast(const float2* b, int n, float v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (b[mid].y >= v) {
            hi = mid;
        } else {
            lo = mid + 1;
        }
    }
    return lo;
}
// Last index i of the nondecreasing lo'[0..n) with lo'[i] <= v (-1 if none).
__device__ __forceinline__ int LastLoAtMost(const float2* b, int n, float v) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (b[mid].x > v) {
            hi = mid;
        } else {
            lo = mid + 1;
        }
    }
    return lo - 1;
}

// One thread per record, records taken in the scene's spatial order (p.order: sorted by the
// screen position of their centroid at scene load), so a block's records fall in few tiles:
// the block counts its (tile, record) pairs in an LDS histogram, reserves each touched
// tile's share of its list with ONE global atomic, then writes the ids. (Per-pair global
// atomics serialise on the busy tiles' counters at the memory side.)
// Longest-processing-time-first launch order of the trace blocks: tiles sorted by their work,
// descending (FULL-stream tiles first, then by the log2 of their candidate count), so the
// heavy tiles start first and the light ones fill in behind them. One block; a counting sort
// over 64 buckets (order within a bucket arbitrary: the frame does not depend on it).
constexpr int kOrderThreads = 1024;
// Counts written by device-scope atomics of the same kernel (the bin kernel's last block) need
// device-scope loads; a later kernel (TileOrderKernel) reads them with plain loads.
template <bool kSameKernel>
__device__ __forceinline__ unsigned LoadCount(const unsigned* c) {
    if constexpr (kSameKernel) {
        return __hip_atomic_load(c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        return *c;
    }
}
template <bool kSameKernel>
__device__ __forceinline__ unsigned TileWorkBucket(const BinParams& p, unsigned t, unsigned large) {
    const unsigned cnt = LoadCount<kSameKernel>(&p.counts[t]);
    if (p.tile_info[t].usable == 0u || cnt > p.capacity) {
        return 63u;
    }
    const unsigned total = cnt + large;
    return total == 0u ? 0u : 32u - __builtin_clz(total);
}
// One block of kThreads threads computes the whole order.
template <bool kSameKernel, int kThreads>
__device__ void TileOrderBlock(const BinParams& p) {
    __shared__ unsigned start[64];
    const int tid = threadIdx.x;
    const unsigned nthreads = kThreads;  // == blockDim.x
    const unsigned tiles = static_cast<unsigned>(p.tiles_x * p.tiles_y);
    const unsigned large = LoadCount<kSameKernel>(&p.counts[tiles]);
    if (tid < 64) {
        start[tid] = 0u;
    }
    // Buckets computed once (counts and tile info loaded once), kept in registers for the
    // placement pass: kMaxBinTiles / blockDim.x tiles per thread at most.
    constexpr int kPer = kMaxBinTiles / kThreads;
    unsigned bucket[kPer];
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const unsigned t = tid + k * nthreads;
        bucket[k] = t < tiles ? TileWorkBucket<kSameKernel>(p, t, large) : 0u;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        if (tid + k * nthreads < tiles) {
            atomicAdd(&start[bucket[k]], static_cast<unsigned>(kParts));
        }
    }
    __syncthreads();
    unsigned first = 0u;  // tiles in heavier buckets
    if (tid < 64) {
        for (int b = 63; b > tid; --b) {
            first += start[b];
        }
    }
    __syncthreads();
    if (tid < 64) {
        start[tid] = first;
    }
    __syncthreads();
#pragma unroll
    for (int k = 0; k < kPer; ++k) {
        const unsigned t = tid + k * nthreads;
        if (t < tiles) {
            const unsigned at = atomicAdd(&start[bucket[k]], static_cast<unsigned>(kParts));
            for (int part = 0; part < kParts; ++part) {
                p.tile_order[at + part] = t * kParts + part;  // trace work items (tile, part)
            }
        }
    }
}

// Monotone tile-column and tile-row bounds of the usable tiles' boxes (lo' = suffix minimum,
// hi' = prefix maximum; both nondecreasing) into out[0 .. nx + ny) (LDS or global). One block
// of >= 4 waves; `scratch` = 2 (nx + ny) LDS words. Ends with a barrier.
__device__ void TileBounds(const BinParams& p, unsigned* scratch, float2* out) {
    const int tid = threadIdx.x;
    const int nthreads = blockDim.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const int nx = p.tiles_x, ny = p.tiles_y;
    const int tiles = nx * ny;
    unsigned* col_lo = scratch;
    unsigned* col_hi = scratch + nx;
    unsigned* row_lo = scratch + 2 * nx;
    unsigned* row_hi = scratch + 2 * nx + ny;
    for (int i = tid; i < nx + ny; i += nthreads) {
        const bool col = i < nx;
        const int j = col ? i : i - nx;
        (col ? col_lo : row_lo)[j] = OrderedBits(__builtin_inff());
        (col ? col_hi : row_hi)[j] = OrderedBits(-__builtin_inff());
    }
    __syncthreads();
    for (int t = tid; t < tiles; t += nthreads) {
        const float4 tb = p.tile_info[t].box;
        if (p.tile_info[t].usable != 0u && tb.x <= tb.y && tb.z <= tb.w) {
            const int c = t % nx, r = t / nx;
            atomicMin(&col_lo[c], OrderedBits(tb.x));
            atomicMax(&col_hi[c], OrderedBits(tb.y));
            atomicMin(&row_lo[r], OrderedBits(tb.z));
            atomicMax(&row_hi[r], OrderedBits(tb.w));
        }
    }
    __syncthreads();
    if (wave == 0) {
        WaveScanOrdered<false>(col_lo, nx, true, lane);
    } else if (wave == 1) {
        WaveScanOrdered<true>(col_hi, nx, false, lane);
    } else if (wave == 2) {
        WaveScanOrdered<false>(row_lo, ny, true, lane);
    } else if (wave == 3) {
        WaveScanOrdered<true>(row_hi, ny, false, lane);
    }
    __syncthreads();
    for (int i = tid; i < nx + ny; i += nthreads) {
        const bool col = i < nx;
        const int j = col ? i : i - nx;
        out[i] = make_float2(FromOrderedBits(col ? col_lo[j] : row_lo[j]), FromOrderedBits(col ? col_hi[j] : row_hi[j]));
    }
    __syncthreads();
}

// One block: the frame's tile bounds, once, for every bin block (a bin block reducing all
// tile infos itself costs O(tiles) L2 reads per block: 0.5 GB per frame at C5).
__global__ __launch_bounds__(1024) void TileBoundsKernel(BinParams p) {
    __shared__ unsigned scratch[2 * kMaxBoundTiles];
    TileBounds(p, scratch, p.bounds);
}

__global__ __launch_bounds__(kBinThreads) void BinTrianglesKernel(BinParams p) {
    __shared__ float2 b[kMaxBoundTiles];
    __shared__ unsigned hist[kMaxBinTiles];
    const int tid = threadIdx.x;
    const int nx = p.tiles_x, ny = p.tiles_y;
    const int tiles = nx * ny;

    // Prologue: the monotone tile-column and tile-row bounds -- precomputed once per frame by
    // TileBoundsKernel (p.bounds), or reduced here by every block (SRT_TILE_BOUNDS=0).
    if (p.bounds != nullptr) {
        for (int i = tid; i < nx + ny; i += kBinThreads) {
            b[i] = p.bounds[i];
        }
    } else {
        TileBounds(p, hist, b);
    }
    __syncthreads();
    for (int t = tid; t < tiles; t += kBinThreads) {
        hist[t] = 0u;
    }

    // This thread's record: its tile range and the tiles of it that pass (bit k = tile
    // (r0 + k / w, c0 + k % w) of the range, at most kLargeTiles of them).
    const unsigned i = blockIdx.x * kBinThreads + tid;  // spatial-order position (list entry)
    unsigned mask = 0u;
    int c0 = 0, r0 = 0, w = 1;
    if (i < p.n) {
        const CullRecord cr = p.cull[i];
        const float4 sb = cr.sb;
        if (sb.x <= sb.y && sb.z <= sb.w && (p.exp & 1u) == 0u) {  // else disabled: empty box
            // Any tile (c, r) whose box overlaps sb has hi'[c] >= hi[c] >= sb.xlo and
            // lo'[c] <= lo[c] <= sb.xhi, so c lies in [c0, c1]; rows likewise.
            c0 = FirstHiAtLeast(b, nx, sb.x);
            const int c1 = LastLoAtMost(b, nx, sb.y);
            r0 = FirstHiAtLeast(b + nx, ny, sb.z);
            const int r1 = LastLoAtMost(b + nx, ny, sb.w);
            w = c1 - c0 + 1;
            const int h = r1 - r0 + 1;
            if (w > 0 && h > 0 && (p.exp & 2u) == 0u) {
                if (w * h > kLargeTiles) {
                    p.large_list[atomicAdd(&p.counts[tiles], 1u)] = i;
                } else {
                    const Record rec{cr.a.x, cr.a.y, cr.a.z, cr.a.w, cr.b.x, cr.b.y, cr.b.z, cr.b.w, cr.x.x};
                    for (int k = 0; k < w * h; ++k) {
                        const TileInfo ti = p.tile_info[(r0 + k / w) * nx + c0 + k % w];
                        const Box tb{ti.box.x, ti.box.y, ti.box.z, ti.box.w};
                        if (ti.usable != 0u && ScreenBoxOverlaps(tb, sb) && BoxMayHit(tb, rec)) {
                            mask |= 1u << k;
                        }
                    }
                }
            }
        }
    }
    __syncthreads();  // histogram zeroed
    for (unsigned m = mask; m != 0u; m &= m - 1u) {
        const int k = __builtin_ctz(m);
        atomicAdd(&hist[(r0 + k / w) * nx + c0 + k % w], 1u);
    }
    __syncthreads();
    for (int t = tid; t < tiles; t += kBinThreads) {
        const unsigned h = hist[t];
        if (h != 0u) {
            hist[t] = (p.exp & 4u) ? 0u : atomicAdd(&p.counts[t], h);  // this block's base in the list
        }
    }
    __syncthreads();
    for (unsigned m = mask; m != 0u; m &= m - 1u) {
        const int k = __builtin_ctz(m);
        const unsigned t = static_cast<unsigned>((r0 + k / w) * nx + c0 + k % w);
        const unsigned at = atomicAdd(&hist[t], 1u);
        if (at < p.capacity) {
            p.lists[static_cast<size_t>(t) * p.capacity + at] = i;
        }
    }
    // The last block to finish computes the trace launch order from the final list counts.
    // Every count update of a block is an atomic whose returned value the block consumed
    // before this barrier, so it has been performed at the device coherence point; the last
    // block reads the counts with device-scope atomic loads (no L2-wide fences needed).
    __shared__ unsigned last;
    if (p.order_in_bin == 0u) {
        return;
    }
    __syncthreads();
    if (tid == 0) {
        last = atomicAdd(&p.sync[0], 1u) == gridDim.x - 1u ? 1u : 0u;
    }
    __syncthreads();
    if (last != 0u) {
        TileOrderBlock<true, kBinThreads>(p);
        if (tid == 0) {
            p.sync[0] = 0u;  // ready for the next frame (the kernel boundary orders it)
        }
    }
}

// Standalone order (a band with no records: the bin kernel, which normally computes the
// order in its last block, is not launched).
__global__ __launch_bounds__(kOrderThreads) void TileOrderKernel(BinParams p) {
    TileOrderBlock<false, kOrderThreads>(p);
}

// Candidate source of a tile: LIST (binned, usable box, list complete): the tile's list then
// the large list; FULL (no bins, an unusable tile box, or an overflowed list): every record.
__device__ __forceinline__ CullSource TileSource(const TraceParams& p, const TileInfo& ti, unsigned tile) {
    CullSource src{nullptr, nullptr, 0u, 0u, 0u, 0u, p.n_pad / kStreamStep};
    if (p.tile_info == nullptr) {
        return src;
    }
    const unsigned cnt = p.bin_counts[tile];
    if (ti.usable != 0u && cnt <= p.bin_capacity) {
        src.list = p.bin_lists + static_cast<size_t>(tile) * p.bin_capacity;
        src.list2 = p.large_list;
        src.count1 = cnt;
        src.end = cnt + p.bin_counts[p.tiles];
    }
    return src;
}

// Rays of a regular tile (every offset equal to (ox, oy), bit for bit): GenerateRays'
// expressions without reading the offsets.
template <int R>
__device__ __forceinline__ void UniformRays(const TraceParams& p, int x, int y_in_block, float ox, float fy_rows,
                                            Rays<R>& s, Box& box) {
    const int xc = min(x, p.width - 1);
    const float fx = (static_cast<float>(xc) + ox) / p.wf;
    box = Box{__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()};
#pragma unroll
    for (int r = 0; r < R; ++r) {
        s.fx[r] = fx;
        // Row r's fy is wave-uniform: lane (y0 - row0) + r of fy_rows computed it (the same
        // expression, (float(row_begin + yc) + oy) / hf), one division per lane instead of R.
        s.fy[r] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fy_rows), y_in_block + r));
        s.bt[r] = __builtin_inff();
        s.bi[r] = -1;
        box.xlo = fminf(box.xlo, s.fx[r]);
        box.xhi = fmaxf(box.xhi, s.fx[r]);
        box.ylo = fminf(box.ylo, s.fy[r]);
        box.yhi = fmaxf(box.yhi, s.fy[r]);
    }
}

#ifndef SRT_TRACE_OCC
#define SRT_TRACE_OCC 4
#endif
template <int W>
__global__ __launch_bounds__(kWave * W, SRT_TRACE_OCC) void TraceCullKernel(TraceParams p) {
    using S = CullShape<W>;
    constexpr int R = S::kR;
    __shared__ CullShared<W> sh;
    // Block = one part (kBlockRows rows) of a cull tile (kTileRows rows); launched in the
    // tile order's work order when the frame is binned.
    const unsigned linear = blockIdx.y * gridDim.x + blockIdx.x;
    const unsigned item = p.tile_order != nullptr ? p.tile_order[linear] : linear;
    const unsigned tile = item / kParts;
    const int tx = static_cast<int>(tile % static_cast<unsigned>(p.tiles_x));
    const int ty = static_cast<int>(tile / static_cast<unsigned>(p.tiles_x));
    const int row0 = ty * kTileRows + static_cast<int>(item % kParts) * kBlockRows;  // band row of the block
    if (row0 >= p.row_count) {
        return;  // the last tile row's empty part
    }
    const bool binned = p.tile_info != nullptr;
    TileInfo ti{};
    if (binned) {
        ti = p.tile_info[tile];
    }
    const CullSource src = TileSource(p, ti, tile);
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    const int x = tx * kWave + lane;
    const int y0 = row0 + wave * R;
    Rays<R> s;
    Box lane_box;
    bool same = true;
    // Raster walks: lane = column (fx), lanes 0..kBlockRows-1 carry the block's rows' fy (the
    // GenerateRays expression; bit-identical since every ray has the same offset).
    float fy_lane = __builtin_nanf("");
    const bool uniform_rays = binned && ti.regular != 0u;
    if (uniform_rays) {
        if (lane < kBlockRows) {
            const int yc = min(row0 + lane, p.row_count - 1);
            fy_lane = (static_cast<float>(p.row_begin + yc) + ti.oy) / p.hf;
        }
        UniformRays<R>(p, x, wave * R, ti.ox, fy_lane, s, lane_box);
    } else {
        same = GenerateRays<R>(p, x, y0, s, lane_box);
    }
    const Box wb = WaveReduceBox(lane_box);
    // Raster walk eligibility: every ray of the block has the tile's first sample offset (bit
    // pattern), so fx depends on the column only and fy on the row only.
    bool regular = true;
    float oy0;
    if (binned) {
        regular = ti.regular != 0u;
        oy0 = ti.oy;
    } else {
        const int x0 = min(tx * kWave, p.width - 1);
        const float2 o0 = p.offsets[static_cast<size_t>(row0) * p.width + x0];
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
    Box bb = sh.wave_box[0];  // the block's ray box
#pragma unroll
    for (int w = 1; w < W; ++w) {
        const Box o = sh.wave_box[w];
        bb = Box{fminf(bb.xlo, o.xlo), fmaxf(bb.xhi, o.xhi), fminf(bb.ylo, o.ylo), fmaxf(bb.yhi, o.yhi)};
    }
    const bool list = src.list != nullptr;
    const bool raster = sh.regular != 0u && p.allow_raster != 0;
    const bool shared_fx = sh.shared_fx != 0u;
    const float fx_lane = s.fx[0];
    if (!uniform_rays && lane < kBlockRows) {
        const int yc = min(row0 + lane, p.row_count - 1);
        fy_lane = (static_cast<float>(p.row_begin + yc) + oy0) / p.hf;
    }
    if (raster) {
        if (list) {
            PacketWalk<W>(p, sh, s, bb, fx_lane, fy_lane, src, tx, row0);
        } else {
            CullWalk<W, true, true, false>(p, sh, s, bb, wb, fx_lane, fy_lane, src, tile);
        }
    } else if (shared_fx) {
        if (list) {
            CullWalk<W, true, false, true>(p, sh, s, bb, wb, fx_lane, fy_lane, src, tile);
        } else {
            CullWalk<W, true, false, false>(p, sh, s, bb, wb, fx_lane, fy_lane, src, tile);
        }
    } else {
        if (list) {
            CullWalk<W, false, false, true>(p, sh, s, bb, wb, fx_lane, fy_lane, src, tile);
        } else {
            CullWalk<W, false, false, false>(p, sh, s, bb, wb, fx_lane, fy_lane, src, tile);
        }
    }
    ShadeAndStore<R>(p, x, y0, s);
}

// ---------------------------------------------------------------------------------------
// BVH variant: primary rays share the eye, so the closest-hit search
// is a 2-D query over the records' screen boxes. The tree is implicit and 8 wide over the
// cull records in the scene's spatial (Morton) order -- no sort, no topology arrays; only the
// node boxes and depth bounds are refitted per frame (BvhLeafKernel: leaves + level 1 in one
// pass; BvhUpperKernel: one block for the remaining levels). Traversal is wave-uniform: a
// wave owns a 16 x 16 square of rays (4 per lane), tests child boxes against the wave's ray
// box, keeps its stack in LDS and reads node data with wave-uniform loads; at a leaf every
// ray runs the exact test on the records that pass the wave-box tests (ExactTestAnyOrder:
// (t, id) minimum in any order). A child whose depth lower bound exceeds the largest best t
// of the wave's rays is skipped: it can neither win nor tie at any of them. Bit-identical to
// brute force by the same arguments as the cull variant.
// ---------------------------------------------------------------------------------------
struct BvhParams {
    const CullRecord* __restrict__ cull;  // records in spatial order
    float4* __restrict__ boxes;           // all levels
    float* __restrict__ tlo;              // all levels
    BvhLayout layout;
    unsigned n;
};

// Exact lower bound of the t any pixel of the box can compute for a record. With u = 2^-24
// and M = sum_k (|c0_k| + max|fx| |cx_k| + max|fy| |cy_k|) over the box: each computed edge
// function (two fma roundings) is within 2.01 u M_k of the exact affine E_k; a hit has all
// computed E_k >= 0, so the computed det = (E_A + E_B) + E_C (two rounded adds of nonnegative
// terms) is <= (1 + 2.01 u) (det_exact + 2.01 u M), and det_exact = S0 + Sx fx + Sy fy is at
// most its value at the box corner picked by the signs of (Sx, Sy). Evaluated in double with
// a 1e-15 relative pad for the double roundings; then every hit in the box has det <= det_max
// and t = fl(vol / det) >= round_down(vol / det_max) (vol > 0; rounding is monotone).
// No hit possible: +inf. Unbounded box or non-finite data: 0 (never culls).
__device__ __forceinline__ float DepthLowerBound(const float4& box, const CullRecord& r) {
    constexpr double u = 0x1p-24;
    const float c0[3] = {r.a.x, r.a.w, r.b.z}, cx[3] = {r.a.y, r.b.x, r.b.w}, cy[3] = {r.a.z, r.b.y, r.x.x};
    double s0 = 0.0, sx = 0.0, sy = 0.0, m0 = 0.0, mx = 0.0, my = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        s0 += c0[k];
        sx += cx[k];
        sy += cy[k];
        m0 += fabs(static_cast<double>(c0[k]));
        mx += fabs(static_cast<double>(cx[k]));
        my += fabs(static_cast<double>(cy[k]));
    }
    const double fx = sx >= 0.0 ? box.y : box.x;
    const double fy = sy >= 0.0 ? box.w : box.z;
    const double ax = fmax(fabs(static_cast<double>(box.x)), fabs(static_cast<double>(box.y)));
    const double ay = fmax(fabs(static_cast<double>(box.z)), fabs(static_cast<double>(box.w)));
    const double m = m0 + ax * mx + ay * my;
    const double det = s0 + sx * fx + sy * fy;
    const double x = det + 1e-15 * (fabs(det) + m) + 2.01 * u * m + 1e-300;
    if (!(x > 0.0)) {
        return x <= 0.0 ? __builtin_inff() : 0.f;
    }
    const double t = static_cast<double>(r.x.y) / (x * (1.0 + 2.01 * u) * (1.0 + 1e-15));
    return t == t ? __double2float_rd(t) : 0.f;
}

__device__ __forceinline__ float4 BoxUnion(const float4& a, const float4& b) {
    return make_float4(fminf(a.x, b.x), fmaxf(a.y, b.y), fminf(a.z, b.z), fmaxf(a.w, b.w));
}

// Leaves (one thread each) and level 1 (the first 32 threads of each 256-thread block).
__global__ __launch_bounds__(256) void BvhLeafKernel(BvhParams p) {
    __shared__ float4 box[256];
    __shared__ float lo[256];
    const unsigned tid = threadIdx.x;
    const unsigned leaf = blockIdx.x * 256 + tid;
    const unsigned nleaf = p.layout.count[0];
    float4 b = make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff());
    float t = __builtin_inff();
    if (leaf < nleaf) {
        const unsigned r1 = min(p.n, (leaf + 1) * kBvhWidth);
        for (unsigned r = leaf * kBvhWidth; r < r1; ++r) {
            const CullRecord cr = p.cull[r];
            if (cr.sb.x <= cr.sb.y && cr.sb.z <= cr.sb.w) {  // else disabled: never hit
                b = BoxUnion(b, cr.sb);
                t = fminf(t, DepthLowerBound(cr.sb, cr));
            }
        }
        p.boxes[p.layout.offset[0] + leaf] = b;
        p.tlo[p.layout.offset[0] + leaf] = t;
    }
    box[tid] = b;
    lo[tid] = t;
    __syncthreads();
    if (p.layout.levels > 1 && tid < 256 / kBvhWidth) {
        const unsigned node = blockIdx.x * (256 / kBvhWidth) + tid;
        if (node < p.layout.count[1]) {
            float4 u = box[tid * kBvhWidth];
            float v = lo[tid * kBvhWidth];
#pragma unroll
            for (int c = 1; c < kBvhWidth; ++c) {
                u = BoxUnion(u, box[tid * kBvhWidth + c]);
                v = fminf(v, lo[tid * kBvhWidth + c]);
            }
            p.boxes[p.layout.offset[1] + node] = u;
            p.tlo[p.layout.offset[1] + node] = v;
        }
    }
}

// Levels 2.. in one block, level by level (one workgroup: the barrier orders a level's
// writes before the next level's reads).
__global__ __launch_bounds__(1024) void BvhUpperKernel(BvhParams p) {
    for (unsigned L = 2; L < p.layout.levels; ++L) {
        const unsigned below = p.layout.offset[L - 1], nb = p.layout.count[L - 1];
        for (unsigned i = threadIdx.x; i < p.layout.count[L]; i += blockDim.x) {
            float4 u = make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff());
            float v = __builtin_inff();
            const unsigned c1 = min(nb, (i + 1) * kBvhWidth);
            for (unsigned c = i * kBvhWidth; c < c1; ++c) {
                u = BoxUnion(u, p.boxes[below + c]);
                v = fminf(v, p.tlo[below + c]);
            }
            p.boxes[p.layout.offset[L] + i] = u;
            p.tlo[p.layout.offset[L] + i] = v;
        }
        __threadfence_block();
        __syncthreads();
    }
}

constexpr int kBvhWaves = 4;  // block = 4 waves side by side, 64 columns x 16 rows
constexpr int kBvhRows = 4;   // rays per lane (lane = one column of a 16 x 16 wave square)
// Per-wave traversal stack: a pop pushes at most kBvhWidth children, so depth <= 7 L + 1 for
// L levels; 11 levels cover 8^11 > 2^31 records (the scene-file limit).
constexpr int kBvhStack = (kBvhWidth - 1) * 11 + 1;

struct BvhTraceArgs {
    TraceParams t;
    const float4* __restrict__ boxes;
    const float* __restrict__ tlo;
    BvhLayout layout;
};

// Largest best t over the wave's rays; +inf while any of them has no hit.
template <int R>
__device__ __forceinline__ float WaveMaxBestT(const Rays<R>& s) {
    float m = s.bt[0];
#pragma unroll
    for (int r = 1; r < R; ++r) {
        m = fmaxf(m, s.bt[r]);
    }
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        m = fmaxf(m, __shfl_xor(m, o));
    }
    return m;
}

template <bool SHARED>
__device__ __forceinline__ void BvhWalk(const BvhTraceArgs& a, Rays<kBvhRows>& s, const Box& wb, bool wb_usable,
                                        unsigned* stack) {
    const TraceParams& p = a.t;
    const int lane = threadIdx.x & (kWave - 1);
    const unsigned top = a.layout.levels - 1;
    if (lane == 0) {
        stack[0] = top << 28;
    }
    int sp = 1;
    // Depth cut, only with a usable wave box: the screen boxes (and the depth bounds computed
    // over them) bound only rays with |fx|, |fy| <= kScreenBoxRange.
    float wave_t = __builtin_inff();
    while (sp > 0) {
        --sp;
        const unsigned e = __builtin_amdgcn_readfirstlane(stack[sp]);
        const unsigned level = e >> 28, idx = e & 0x0FFFFFFFu;
        if (level == 0) {
            const unsigned r1 = min(p.n, (idx + 1) * kBvhWidth);
            bool tested = false;
            for (unsigned r = idx * kBvhWidth; r < r1; ++r) {
                const CullRecord cr = p.cull[r];
                const Record q{cr.a.x, cr.a.y, cr.a.z, cr.a.w, cr.b.x, cr.b.y, cr.b.z, cr.b.w, cr.x.x};
                if ((wb_usable && !ScreenBoxOverlaps(wb, cr.sb)) || !BoxMayHit(wb, q)) {
                    continue;
                }
                ExactTestAnyOrder<kBvhRows, SHARED>(s, q, cr.x.y, __float_as_int(cr.x.z));
                tested = true;
            }
            if (tested && wb_usable) {
                wave_t = WaveMaxBestT<kBvhRows>(s);
            }
            continue;
        }
        const unsigned below = a.layout.offset[level - 1], nb = a.layout.count[level - 1];
        const unsigned c0 = idx * kBvhWidth;
        // The kept children sorted by depth bound, largest first (a fixed 19-comparator
        // network on wave-uniform values), then pushed in that order: the nearest pops first,
        // so the depth cut tightens early. Not kept: key -1 (bounds are >= 0).
        float kt[kBvhWidth];
        unsigned ki[kBvhWidth];
#pragma unroll
        for (int j = 0; j < kBvhWidth; ++j) {
            const unsigned c = c0 + j;
            bool keep = false;
            float ct = 0.f;
            if (c < nb) {
                const float4 cb = a.boxes[below + c];
                ct = a.tlo[below + c];
                keep = wb_usable ? (ScreenBoxOverlaps(wb, cb) && !(ct > wave_t)) : true;
            }
            kt[j] = keep ? ct : -1.f;
            ki[j] = c;
        }
        auto ce = [&](int i, int j) {
            if (kt[i] < kt[j]) {
                const float t = kt[i];
                kt[i] = kt[j];
                kt[j] = t;
                const unsigned u = ki[i];
                ki[i] = ki[j];
                ki[j] = u;
            }
        };
        ce(0, 2); ce(1, 3); ce(4, 6); ce(5, 7);
        ce(0, 4); ce(1, 5); ce(2, 6); ce(3, 7);
        ce(0, 1); ce(2, 3); ce(4, 5); ce(6, 7);
        ce(2, 4); ce(3, 5);
        ce(1, 4); ce(3, 6);
        ce(1, 2); ce(3, 4); ce(5, 6);
#pragma unroll
        for (int j = 0; j < kBvhWidth; ++j) {
            if (kt[j] >= 0.f) {
                if (lane == 0) {
                    stack[sp] = ((level - 1) << 28) | ki[j];
                }
                ++sp;
            }
        }
    }
}

__global__ __launch_bounds__(kWave * kBvhWaves) void TraceBvhKernel(BvhTraceArgs a) {
    __shared__ unsigned stacks[kBvhWaves][kBvhStack];
    constexpr int R = kBvhRows;
    const TraceParams& p = a.t;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
    // Wave footprint: a 16 x 16 square of rays (the fewest records overlap a square); lane =
    // column lane % 16, rows (lane / 16) * 4 .. + 3.
    const int x = blockIdx.x * kWave + wave * 16 + (lane & 15);
    const int y0 = blockIdx.y * (4 * R) + (lane >> 4) * R;
    Rays<R> s;
    Box lane_box;
    const bool same = GenerateRays<R>(p, x, y0, s, lane_box);
    const Box wb = WaveReduceBox(lane_box);
    if (p.n != 0u && static_cast<int>(blockIdx.y) * 4 * R < p.row_count) {
        if (__all(same)) {
            BvhWalk<true>(a, s, wb, ScreenBoxUsable(wb), stacks[wave]);
        } else {
            BvhWalk<false>(a, s, wb, ScreenBoxUsable(wb), stacks[wave]);
        }
    }
    ShadeAndStore<R>(p, x, y0, s);
}

// Boolean env switch ("0" = off), for measurement of alternatives.
bool EnvFlag(const char* name, bool dflt) {
    const char* v = std::getenv(name);
    return v == nullptr || *v == '\0' ? dflt : std::strcmp(v, "0") != 0;
}

// Waves per trace block; env SRT_CULL_WAVES = 4, 8 or 16 (default 4), for measurement.
int CullWavesFromEnv() {
    const char* v = std::getenv("SRT_CULL_WAVES");
    if (v != nullptr && (std::strcmp(v, "8") == 0 || std::strcmp(v, "16") == 0)) {
        return std::atoi(v);
    }
    return 4;
}

// ML_FLOAT16 images: 4 elements per thread (8-B half / 16-B float vectors), scalar tail.
__global__ __launch_bounds__(256) void FloatToHalfKernel(const float* __restrict__ src, _Float16* __restrict__ dst,
                                                         std::size_t count) {
    const std::size_t i = (static_cast<std::size_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
    if (i + 4 <= count) {
        const float4 v = *reinterpret_cast<const float4*>(src + i);
        typedef _Float16 H4 __attribute__((ext_vector_type(4)));
        *reinterpret_cast<H4*>(dst + i) = H4{static_cast<_Float16>(v.x), static_cast<_Float16>(v.y),
                                             static_cast<_Float16>(v.z), static_cast<_Float16>(v.w)};
    } else {
        for (std::size_t k = i; k < count; ++k) {
            dst[k] = static_cast<_Float16>(src[k]);
        }
    }
}
__global__ __launch_bounds__(256) void HalfToFloatKernel(const _Float16* __restrict__ src, float* __restrict__ dst,
                                                         std::size_t count) {
    const std::size_t i = (static_cast<std::size_t>(blockIdx.x) * blockDim.x + threadIdx.x) * 4;
    for (std::size_t k = i; k < i + 4 && k < count; ++k) {
        dst[k] = static_cast<float>(src[k]);
    }
}

// Launch on `stream`; with timing events, through hipExtLaunchKernelGGL so that the events
// take the dispatch packet's own start / end timestamps (no extra stream packets).
template <class K, class P>
void Launch(K kernel, dim3 grid, dim3 block, hipStream_t stream, hipEvent_t start, hipEvent_t stop, const P& p) {
    if (start != nullptr || stop != nullptr) {
        hipExtLaunchKernelGGL(kernel, grid, block, 0, stream, start, stop, 0, p);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, 0, stream, p);
    }
}

}  // namespace

#ifdef SRT_DIAG
hipError_t DiagRead(void* host, std::size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_srt_diag), bytes < sizeof(g_srt_diag) ? bytes : sizeof(g_srt_diag));
}
#endif

namespace {
PrepareParams MakePrepareParams(const float* d_vertices, const unsigned* d_rank, std::uint64_t n, const Frame& frame,
                                float* d_edges) {
    PrepareParams p{};
    p.vertices = d_vertices;
    p.rank = d_rank;
    p.edges = reinterpret_cast<float4*>(d_edges);
    p.screen_boxes = reinterpret_cast<float4*>(d_edges) + PaddedTriangleCount(n) / kTileTriangles * kTileFloat4;
    p.qboxes = reinterpret_cast<uint2*>(p.screen_boxes + PaddedTriangleCount(n));
    p.cull = reinterpret_cast<CullRecord*>(p.qboxes + PaddedTriangleCount(n));
    p.normals = reinterpret_cast<float4*>(p.cull + PaddedTriangleCount(n));
    p.n = static_cast<unsigned>(n);
    p.n_pad = static_cast<unsigned>(PaddedTriangleCount(n));
    for (int k = 0; k < 3; ++k) {
        p.origin[k] = frame.origin[k];
        p.base[k] = frame.base[k];
        p.du[k] = frame.du[k];
        p.dv[k] = frame.dv[k];
    }
#ifdef SRT_DIAG
    if (const char* e = std::getenv("SRT_EXP")) {
        p.exp = static_cast<unsigned>(std::strtoul(e, nullptr, 0));
    }
#endif
    return p;
}
}  // namespace

hipError_t LaunchFloatToHalf(const float* src, std::uint16_t* dst, std::size_t count, hipStream_t stream) {
    if (count == 0) {
        return hipSuccess;
    }
    const unsigned blocks = static_cast<unsigned>((count + 1023) / 1024);
    hipLaunchKernelGGL(FloatToHalfKernel, dim3(blocks), dim3(256), 0, stream, src, reinterpret_cast<_Float16*>(dst),
                       count);
    return hipGetLastError();
}

hipError_t LaunchHalfToFloat(const std::uint16_t* src, float* dst, std::size_t count, hipStream_t stream) {
    if (count == 0) {
        return hipSuccess;
    }
    const unsigned blocks = static_cast<unsigned>((count + 1023) / 1024);
    hipLaunchKernelGGL(HalfToFloatKernel, dim3(blocks), dim3(256), 0, stream,
                       reinterpret_cast<const _Float16*>(src), dst, count);
    return hipGetLastError();
}

hipError_t LaunchPrepare(const float* d_vertices, const unsigned* d_rank, std::uint64_t n, const Frame& frame,
                         float* d_edges, hipStream_t stream, hipEvent_t ev_begin, hipEvent_t ev_end) {
    const PrepareParams p = MakePrepareParams(d_vertices, d_rank, n, frame, d_edges);
    const unsigned blocks = (p.n_pad + 255) / 256;
    Launch(PrepareKernel, dim3(blocks), dim3(256), stream, ev_begin, ev_end, p);
    return hipGetLastError();
}

BvhLayout MakeBvhLayout(std::uint64_t n) {
    BvhLayout l;
    std::uint64_t below = n == 0 ? 1 : n;
    unsigned offset = 0;
    do {
        const std::uint64_t c = (below + kBvhWidth - 1) / kBvhWidth;
        if (l.levels == kBvhMaxLevels) {
            throw std::runtime_error("BVH too deep");
        }
        l.count[l.levels] = static_cast<unsigned>(c);
        l.offset[l.levels] = offset;
        offset += static_cast<unsigned>(c);
        ++l.levels;
        below = c;
    } while (below > 1);
    l.nodes = offset;
    return l;
}

namespace {
std::size_t BvhBoxBytes(const BvhLayout& l) { return (static_cast<std::size_t>(l.nodes) * 16 + 255) / 256 * 256; }
}  // namespace

std::size_t BvhBytes(std::uint64_t n) {
    const BvhLayout l = MakeBvhLayout(n);
    return BvhBoxBytes(l) + (static_cast<std::size_t>(l.nodes) * 4 + 255) / 256 * 256;
}

std::size_t CullTiles(std::size_t width, std::size_t row_count) {
    return (width + kWave - 1) / kWave * ((row_count + kTileRows - 1) / kTileRows);
}

bool CullBinnable(std::size_t width, std::size_t row_count) {
    const std::size_t tx = (width + kWave - 1) / kWave, ty = (row_count + kTileRows - 1) / kTileRows;
    return tx + ty <= kMaxBoundTiles && tx * ty <= kMaxBinTiles;
}

unsigned CullBinCapacity(std::uint64_t n, std::size_t tiles) {
    const std::uint64_t n_pad = PaddedTriangleCount(n);
    std::uint64_t cap = tiles == 0 ? n_pad : 64 * n_pad / tiles;
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

namespace {
struct BinSizes {
    std::size_t info, counts, lists, large, order, sync, bounds;
};
BinSizes CullBinSizes(std::uint64_t n, std::size_t width, std::size_t row_count) {
    const std::size_t tx = (width + kWave - 1) / kWave, ty = (row_count + kTileRows - 1) / kTileRows;
    const std::size_t tiles = tx * ty;
    const auto al = [](std::size_t b) { return (b + 255) / 256 * 256; };
    BinSizes z;
    z.info = al(tiles * sizeof(TileInfo));
    z.counts = al((tiles + 1) * 4);
    z.lists = al(tiles * static_cast<std::size_t>(CullBinCapacity(n, tiles)) * 4);
    z.large = al(PaddedTriangleCount(n) * 4);
    z.order = al(tiles * kParts * 4);
    z.sync = al(4);
    z.bounds = al((tx + ty) * 8);
    return z;
}
}  // namespace

std::size_t CullBinBytes(std::uint64_t n, std::size_t width, std::size_t row_count) {
    const BinSizes z = CullBinSizes(n, width, row_count);
    return z.info + z.counts + z.lists + z.large + z.order + z.sync + z.bounds;
}

CullBins CullBinLayout(void* base, std::uint64_t n, std::size_t width, std::size_t row_count) {
    const BinSizes z = CullBinSizes(n, width, row_count);
    unsigned char* w = static_cast<unsigned char*>(base);
    CullBins b{};
    b.tile_info = w;
    w += z.info;
    b.counts = reinterpret_cast<unsigned*>(w);
    w += z.counts;
    b.lists = reinterpret_cast<unsigned*>(w);
    w += z.lists;
    b.large_list = reinterpret_cast<unsigned*>(w);
    w += z.large;
    b.tile_order = reinterpret_cast<unsigned*>(w);
    w += z.order;
    b.sync = reinterpret_cast<unsigned*>(w);
    w += z.sync;
    b.bounds = w;
    b.tiles = CullTiles(width, row_count);
    b.capacity = CullBinCapacity(n, b.tiles);
    return b;
}

hipError_t LaunchTrace(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_albedo,
                       const Frame& frame, const float background[3], const BandArgs& band, int variant,
                       const CullBins* bins, hipStream_t stream, const StageEvents* events,
                       const unsigned* prepare_rank, void* bvh) {
    if (band.row_count == 0 || band.width == 0) {
        return hipSuccess;
    }
    const StageEvents ev = events != nullptr ? *events : StageEvents{};
    const bool fuse_prepare =
        prepare_rank != nullptr && variant == kTraceCull && bins != nullptr && EnvFlag("SRT_FUSE_PREPARE", true);
    if (prepare_rank != nullptr && !fuse_prepare) {
        const hipError_t e = LaunchPrepare(d_vertices, prepare_rank, n, frame, const_cast<float*>(d_edges), stream,
                                           ev.prep_begin, ev.prep_end);
        if (e != hipSuccess) {
            return e;
        }
    }
    TraceParams p{};
    p.edges = reinterpret_cast<const float4*>(d_edges);
    p.screen_boxes = reinterpret_cast<const float4*>(d_edges) + PaddedTriangleCount(n) / kTileTriangles * kTileFloat4;
    p.qboxes = reinterpret_cast<const uint2*>(p.screen_boxes + PaddedTriangleCount(n));
    p.cull = reinterpret_cast<const CullRecord*>(p.qboxes + PaddedTriangleCount(n));
    p.normals = reinterpret_cast<const float4*>(p.cull + PaddedTriangleCount(n));
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
    }
    p.wf = static_cast<float>(band.width);
    p.hf = static_cast<float>(band.height);
    for (int k = 0; k < 3; ++k) {
        p.base[k] = frame.base[k];
        p.du[k] = frame.du[k];
        p.dv[k] = frame.dv[k];
        p.bg[k] = background[k];
    }
    p.n = static_cast<unsigned>(n);
    const unsigned gx = static_cast<unsigned>((band.width + kWave - 1) / kWave);
    if (variant == kTraceBvh) {
        if (bvh == nullptr) {
            return hipErrorInvalidValue;
        }
        BvhParams bp{};
        bp.cull = p.cull;
        bp.layout = MakeBvhLayout(n);
        bp.boxes = static_cast<float4*>(bvh);
        bp.tlo = reinterpret_cast<float*>(static_cast<unsigned char*>(bvh) + BvhBoxBytes(bp.layout));
        bp.n = static_cast<unsigned>(n);
        if (n != 0) {
            Launch(BvhLeafKernel, dim3((bp.layout.count[0] + 255) / 256), dim3(256), stream, ev.bin_begin,
                   bp.layout.levels > 2 ? nullptr : ev.bin_end, bp);
            if (bp.layout.levels > 2) {
                Launch(BvhUpperKernel, dim3(1), dim3(1024), stream, nullptr, ev.bin_end, bp);
            }
        }
        BvhTraceArgs a{};
        a.t = p;
        a.boxes = bp.boxes;
        a.tlo = bp.tlo;
        a.layout = bp.layout;
        constexpr int kRowsPerBlock = kBvhRows * 4;
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerBlock - 1) / kRowsPerBlock);
        Launch(TraceBvhKernel, dim3(gx, gy), dim3(kWave * kBvhWaves), stream, ev.begin, ev.end, a);
        return hipGetLastError();
    }
    if (variant == kTraceScalar) {
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerLane - 1) / kRowsPerLane);
        Launch(TraceScalarKernel, dim3(gx, gy), dim3(kWave), stream, ev.begin, ev.end, p);
    } else if (variant == kTraceCull) {
        const unsigned gy = static_cast<unsigned>((band.row_count + kTileRows - 1) / kTileRows);
        if (bins != nullptr) {
            if (bins->tiles != static_cast<std::size_t>(gx) * gy || !CullBinnable(band.width, band.row_count)) {
                return hipErrorInvalidValue;  // bins sized for another band shape
            }
            BinParams b{};
            b.offsets = p.offsets;
            b.cull = p.cull;
            b.tile_info = static_cast<TileInfo*>(bins->tile_info);
            b.counts = bins->counts;
            b.lists = bins->lists;
            b.large_list = bins->large_list;
            b.tile_order = bins->tile_order;
            b.sync = bins->sync;
            // Tile bounds once per frame (TileBoundsKernel) when the bin blocks' own reductions
            // would cost more: (bin blocks) x (tiles) tile-info reads above 200k (C5: 16M, bin
            // stage 164 -> 75 us; C3: 0.4M, where the extra launch adds ~1 % to one frame's
            // latency but the chip time it saves gives +3 % with frame queues in flight; C2 and
            // small frames: 1k, no extra launch). Env SRT_TILE_BOUNDS=0/1 forces either way.
            {
                const std::uint64_t reads = (n + kBinThreads - 1) / kBinThreads * static_cast<std::uint64_t>(gx) * gy;
                const char* v = std::getenv("SRT_TILE_BOUNDS");
                const bool once = v != nullptr && *v != '\0' ? std::strcmp(v, "0") != 0 : reads > 200000ull;
                b.bounds = once ? static_cast<float2*>(bins->bounds) : nullptr;
            }
            b.capacity = bins->capacity;
            b.n = static_cast<unsigned>(n);
            b.tiles_x = static_cast<int>(gx);
            b.tiles_y = static_cast<int>(gy);
            b.width = p.width;
            b.row_count = p.row_count;
            b.row_begin = p.row_begin;
            b.wf = p.wf;
            b.hf = p.hf;
#ifdef SRT_DIAG
            if (const char* e = std::getenv("SRT_EXP")) {
                b.exp = static_cast<unsigned>(std::strtoul(e, nullptr, 0));
                p.exp = b.exp;
            }
#endif
            if (fuse_prepare) {
                PrepareInfoParams f{};
                f.prep = MakePrepareParams(d_vertices, prepare_rank, n, frame, const_cast<float*>(d_edges));
                f.bin = b;
                f.prep_blocks = (f.prep.n_pad + kBinThreads - 1) / kBinThreads;
                Launch(PrepareInfoKernel, dim3(f.prep_blocks + gx * gy), dim3(kBinThreads), stream, ev.prep_begin,
                       ev.prep_end, f);
            } else {
                Launch(TileInfoKernel, dim3(gx, gy), dim3(kBinThreads), stream, ev.prep_begin, ev.prep_end, b);
            }
            b.order_in_bin = n != 0 && EnvFlag("SRT_ORDER_IN_BIN", false) ? 1u : 0u;
            if (n != 0 && b.bounds != nullptr) {
                Launch(TileBoundsKernel, dim3(1), dim3(1024), stream, ev.bin_begin, nullptr, b);
            }
            if (n != 0) {
                const unsigned blocks = static_cast<unsigned>((n + kBinThreads - 1) / kBinThreads);
                Launch(BinTrianglesKernel, dim3(blocks), dim3(kBinThreads), stream,
                       b.bounds != nullptr ? nullptr : ev.bin_begin,
                       b.order_in_bin != 0u ? ev.bin_end : nullptr, b);
            }
            if (b.order_in_bin == 0u) {
                Launch(TileOrderKernel, dim3(1), dim3(kOrderThreads), stream, n != 0 ? nullptr : ev.bin_begin,
                       ev.bin_end, b);
            }
            p.tile_info = b.tile_info;
            p.order = bins->order;
            p.tile_order = bins->tile_order;
            p.bin_lists = bins->lists;
            p.bin_counts = bins->counts;
            p.large_list = bins->large_list;
            p.bin_capacity = bins->capacity;
        }
        p.tiles_x = static_cast<int>(gx);
        p.tiles = gx * gy;
        // One block per (tile, part): gridDim.x = tile columns, gridDim.y = tile rows x parts.
        const dim3 grid(gx, gy * kParts);
        const int waves = CullWavesFromEnv();
        if constexpr (CullWavesOk(16)) {
            if (waves == 16) {
                Launch(TraceCullKernel<16>, grid, dim3(kWave * 16), stream, ev.begin, ev.end, p);
                return hipGetLastError();
            }
        }
        if constexpr (CullWavesOk(8)) {
            if (waves == 8) {
                Launch(TraceCullKernel<8>, grid, dim3(kWave * 8), stream, ev.begin, ev.end, p);
                return hipGetLastError();
            }
        }
        Launch(TraceCullKernel<4>, grid, dim3(kWave * 4), stream, ev.begin, ev.end, p);
    } else {
        constexpr int kRowsPerBlock = kRowsPerLane * kLdsWaves;
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerBlock - 1) / kRowsPerBlock);
        Launch(TraceLdsKernel, dim3(gx, gy), dim3(kWave * kLdsWaves), stream, ev.begin, ev.end, p);
    }
    return hipGetLastError();
}

}  // namespace srt
