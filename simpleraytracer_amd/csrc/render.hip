// MI355X (gfx950) render kernels: edge-record preparation and the brute-force closest-hit
// trace. The reference has no render code; this file implements the
// north_star stages (a9)-(a12) of SURVEY.md section 8(a) from the canonical math in
// DESIGN.md. Built with -ffp-contract=off: every fused multiply-add below is an explicit
// fmaf, so CPU (oracle/srt_oracle.c) and GPU evaluate bit-identical float expressions.
#include "render.h"

#include <cmath>

namespace srt {
namespace {

constexpr int kWave = 64;
constexpr int kLdsWaves = 4;     // waves per block in the LDS variant
constexpr int kRowsPerLane = 8;  // rays per lane: one image column, 8 consecutive rows

struct TraceParams {
    const float4* __restrict__ edges;
    const float* __restrict__ vertices;
    const float* __restrict__ albedo;
    const float2* __restrict__ offsets;
    float4* __restrict__ out;
    unsigned n_pad;
    int width;
    int row_count;
    int row_begin;
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
    unsigned n;
    unsigned n_pad;
    float origin[3];
    float base[3];
    float du[3];
    float dv[3];
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

// One thread per triangle: origin-relative edge normals nA = B x C, nB = C x A, nC = A x B
// (A, B, C = vertices - eye), signed volume vol = A . nA, orientation normalised so vol > 0,
// then each normal projected onto the affine ray frame: E(fx, fy) = n . (base + fx du + fy dv).
__global__ __launch_bounds__(256) void PrepareKernel(PrepareParams p) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.n_pad) {
        return;
    }
    float4* rec = p.edges + 3ull * i;
    const float qnan = __builtin_nanf("");
    if (i >= p.n) {
        rec[0] = make_float4(qnan, qnan, qnan, qnan);
        rec[1] = make_float4(qnan, qnan, qnan, qnan);
        rec[2] = make_float4(qnan, qnan, 0.f, 0.f);
        return;
    }
    const float* v = p.vertices + 9ull * i;
    const float ax = v[0] - p.origin[0], ay = v[1] - p.origin[1], az = v[2] - p.origin[2];
    const float bx = v[3] - p.origin[0], by = v[4] - p.origin[1], bz = v[5] - p.origin[2];
    const float cx = v[6] - p.origin[0], cy = v[7] - p.origin[1], cz = v[8] - p.origin[2];
    float n[9];
    Cross3(bx, by, bz, cx, cy, cz, n[0], n[1], n[2]);
    Cross3(cx, cy, cz, ax, ay, az, n[3], n[4], n[5]);
    Cross3(ax, ay, az, bx, by, bz, n[6], n[7], n[8]);
    float vol = Dot3(ax, ay, az, n[0], n[1], n[2]);
    if (!(std::isfinite(vol) && vol != 0.f)) {
        rec[0] = make_float4(qnan, qnan, qnan, qnan);
        rec[1] = make_float4(qnan, qnan, qnan, qnan);
        rec[2] = make_float4(qnan, qnan, 0.f, 0.f);
        return;
    }
    if (vol < 0.f) {
#pragma unroll
        for (int k = 0; k < 9; ++k) {
            n[k] = -n[k];
        }
        vol = -vol;
    }
    float c[9];
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const float nx = n[3 * e], ny = n[3 * e + 1], nz = n[3 * e + 2];
        c[3 * e + 0] = Dot3(nx, ny, nz, p.base[0], p.base[1], p.base[2]);
        c[3 * e + 1] = Dot3(nx, ny, nz, p.du[0], p.du[1], p.du[2]);
        c[3 * e + 2] = Dot3(nx, ny, nz, p.dv[0], p.dv[1], p.dv[2]);
    }
    rec[0] = make_float4(c[0], c[1], c[2], c[3]);
    rec[1] = make_float4(c[4], c[5], c[6], c[7]);
    rec[2] = make_float4(c[8], vol, 0.f, 0.f);
}

// Per-lane ray state: R rays sharing one image column.
template <int R>
struct Rays {
    float fx[R];
    float fy[R];
    float bt[R];  // closest t so far (+inf = none)
    int bi[R];    // closest triangle id (-1 = miss)
};

// Test one triangle's edge record against the lane's R rays.
//   hot path:  E_A, E_B, E_C for every ray, candidate iff min(E) >= 0 for some ray
//              (one branch per triangle per wave; candidates are rare)
//   slow path: exact test per ray: all E >= 0, det = (E_A + E_B) + E_C > 0, t = vol / det,
//              strict t < best keeps the lowest id on ties (triangles arrive in id order).
// SHARED: every ray of the lane has the same fx bit pattern, so fma(fx, cx, c0) is one
// value per edge (common-subexpression elimination; the result is bit-identical).
template <int R, bool SHARED>
__device__ __forceinline__ void TestTriangle(Rays<R>& s, float c0A, float cxA, float cyA, float c0B, float cxB,
                                             float cyB, float c0C, float cxC, float cyC, unsigned id,
                                             const float* vol_ptr) {
    float gA[R], gB[R], gC[R];
    if constexpr (SHARED) {
        const float a = fmaf(s.fx[0], cxA, c0A), b = fmaf(s.fx[0], cxB, c0B), c = fmaf(s.fx[0], cxC, c0C);
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gA[r] = a;
            gB[r] = b;
            gC[r] = c;
        }
    } else {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            gA[r] = fmaf(s.fx[r], cxA, c0A);
            gB[r] = fmaf(s.fx[r], cxB, c0B);
            gC[r] = fmaf(s.fx[r], cxC, c0C);
        }
    }
    float m[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const float eA = fmaf(s.fy[r], cyA, gA[r]);
        const float eB = fmaf(s.fy[r], cyB, gB[r]);
        const float eC = fmaf(s.fy[r], cyC, gC[r]);
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
            const float eA = fmaf(s.fy[r], cyA, gA[r]);
            const float eB = fmaf(s.fy[r], cyB, gB[r]);
            const float eC = fmaf(s.fy[r], cyC, gC[r]);
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
// clamped lanes compute but never store).
template <int R>
__device__ __forceinline__ bool GenerateRays(const TraceParams& p, int x, int y0, Rays<R>& s) {
    const int xc = min(x, p.width - 1);
    bool same = true;
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int yc = min(y0 + r, p.row_count - 1);
        const float2 o = p.offsets[static_cast<size_t>(yc) * p.width + xc];
        s.fx[r] = (static_cast<float>(xc) + o.x) / p.wf;
        s.fy[r] = (static_cast<float>(p.row_begin + yc) + o.y) / p.hf;
        s.bt[r] = __builtin_inff();
        s.bi[r] = -1;
        same = same && (__float_as_uint(s.fx[r]) == __float_as_uint(s.fx[0]));
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
// Variant 0: LDS-tiled. Block = 4 waves = 64 columns x 32 rows. Each tile of 256 edge
// records (12 KB) is loaded by the whole block with coalesced 16-B loads into one half of a
// double-buffered LDS ring (24 KB), then every wave walks it with broadcast LDS reads.
// One barrier per tile; the next tile's global loads are in flight during the current one.
// ---------------------------------------------------------------------------------------
using LdsVoidPtr = __attribute__((address_space(3))) void*;

// Copy one 12 KB tile of edge records global -> LDS with LDS-DMA (global_load_lds_dwordx4):
// 12 wave-instructions of 1 KiB per tile, 3 per wave, no VGPR staging; the LDS image is the
// global image (lane-linear). Issued through inline asm so hipcc does not drain it with a
// vmcnt(0) in front of every ds_read of the tile being computed (cdna_hip_programming.md
// section 5 "Pipelining across barriers"); completion is waited for by WaitTile().
__device__ __forceinline__ void StageTile(const float4* __restrict__ src, float4* dst) {
    constexpr int kTileF4 = kTileTriangles * 3;
    constexpr int kPerWave = kTileF4 / (kWave * kLdsWaves);
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x / kWave);
#pragma unroll
    for (int k = 0; k < kPerWave; ++k) {
        const int chunk = (wave * kPerWave + k) * kWave;
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

// Every wave's LDS-DMA done, then the block barrier makes the tile visible to all waves.
__device__ __forceinline__ void WaitTile() {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
}

template <int R, bool SHARED>
__device__ __forceinline__ void WalkTilesLds(const TraceParams& p, float4* lds, Rays<R>& s) {
    constexpr int kTileF4 = kTileTriangles * 3;
    static_assert(kTileF4 % (kWave * kLdsWaves) == 0, "tile must split evenly over the block");
    const unsigned ntiles = p.n_pad / kTileTriangles;
    StageTile(p.edges, lds);
    for (unsigned t = 0; t < ntiles; ++t) {
        const unsigned buf = t & 1u;
        WaitTile();  // tile t landed; every wave is done with tile t-1 (the buffer refilled next)
        if (t + 1 < ntiles) {
            StageTile(p.edges + static_cast<size_t>(t + 1) * kTileF4, lds + (buf ^ 1u) * kTileF4);
        }
        const float4* tile = lds + buf * kTileF4;
        const unsigned id0 = t * kTileTriangles;
#pragma unroll 2
        for (int j = 0; j < kTileTriangles; ++j) {
            const float4 q0 = tile[3 * j];
            const float4 q1 = tile[3 * j + 1];
            const float* q2 = reinterpret_cast<const float*>(tile + 3 * j + 2);
            TestTriangle<R, SHARED>(s, q0.x, q0.y, q0.z, q0.w, q1.x, q1.y, q1.z, q1.w, q2[0], id0 + j, q2 + 1);
        }
    }
}

__global__ __launch_bounds__(kWave * kLdsWaves) void TraceLdsKernel(TraceParams p) {
    // ONE __shared__ object: the double-buffered tile ring plus one flag word at the end
    // (a second LDS object next to LDS-DMA staging makes hipcc wait vmcnt(0) before every
    // ds_read; cdna_hip_programming.md section 5 trap 4(a)).
    __shared__ float4 lds[2 * kTileTriangles * 3 + 1];
    constexpr int R = kRowsPerLane;
    const int lane = threadIdx.x & (kWave - 1);
    const int wave = threadIdx.x / kWave;
    const int x = blockIdx.x * kWave + lane;
    const int y0 = (blockIdx.y * kLdsWaves + wave) * R;
    Rays<R> s;
    const bool same = GenerateRays<R>(p, x, y0, s);
    // Block-uniform choice of loop body (both bodies hold the same barriers).
    unsigned* flag = reinterpret_cast<unsigned*>(lds + 2 * kTileTriangles * 3);
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
    const float* e = reinterpret_cast<const float*>(p.edges);
#pragma unroll 4
    for (unsigned j = 0; j < p.n_pad; ++j) {
        const float* q = e + 12ull * j;
        TestTriangle<R, SHARED>(s, q[0], q[1], q[2], q[3], q[4], q[5], q[6], q[7], q[8], j, q + 9);
    }
}

__global__ __launch_bounds__(kWave) void TraceScalarKernel(TraceParams p) {
    constexpr int R = kRowsPerLane;
    const int x = blockIdx.x * kWave + static_cast<int>(threadIdx.x);
    const int y0 = blockIdx.y * R;
    Rays<R> s;
    const bool same = GenerateRays<R>(p, x, y0, s);
    if (__all(same)) {
        WalkScalar<R, true>(p, s);
    } else {
        WalkScalar<R, false>(p, s);
    }
    ShadeAndStore<R>(p, x, y0, s);
}

}  // namespace

hipError_t LaunchPrepare(const float* d_vertices, std::uint64_t n, const Frame& frame, float* d_edges,
                         hipStream_t stream) {
    PrepareParams p{};
    p.vertices = d_vertices;
    p.edges = reinterpret_cast<float4*>(d_edges);
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

hipError_t LaunchTrace(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_albedo,
                       const Frame& frame, const float background[3], const BandArgs& band, int variant,
                       hipStream_t stream) {
    if (band.row_count == 0 || band.width == 0) {
        return hipSuccess;
    }
    TraceParams p{};
    p.edges = reinterpret_cast<const float4*>(d_edges);
    p.vertices = d_vertices;
    p.albedo = d_albedo;
    p.offsets = reinterpret_cast<const float2*>(band.offsets);
    p.out = reinterpret_cast<float4*>(band.rgba);
    p.n_pad = static_cast<unsigned>(PaddedTriangleCount(n));
    p.width = static_cast<int>(band.width);
    p.row_count = static_cast<int>(band.row_count);
    p.row_begin = static_cast<int>(band.row_begin);
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
    } else {
        constexpr int kRowsPerBlock = kRowsPerLane * kLdsWaves;
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerBlock - 1) / kRowsPerBlock);
        hipLaunchKernelGGL(TraceLdsKernel, dim3(gx, gy), dim3(kWave * kLdsWaves), 0, stream, p);
    }
    return hipGetLastError();
}

}  // namespace srt
