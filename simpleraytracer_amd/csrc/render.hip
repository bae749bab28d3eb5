// MI355X (gfx950) render kernels: edge-record preparation and the brute-force closest-hit
// trace. The reference has no render code; this file implements the
// north_star stages (a9)-(a12) of SURVEY.md section 8(a) from the canonical math in
// DESIGN.md. Built with -ffp-contract=off: every fused multiply-add below is an explicit
// fmaf, so CPU (oracle/srt_oracle.c) and GPU evaluate bit-identical float expressions.
#include "render.h"
#include "screen_box.h"

#include <hip/hip_ext.h>

#include <cmath>
#include <cstdlib>
#include <cstdio>
#include <algorithm>
#include <cstring>
#include <stdexcept>
#include <string>
#include <type_traits>

namespace srt {

#ifdef SRT_DIAG
// Diagnostic build only (make diag): per-block phase cycle counts of the cull kernel.
// [block][0] stream cycles, [1] gather cycles, [2] filter+walk cycles, [3] block survivors,
// [4] packets (packet walk) / wave-0 survivors walked (stream walk), [5] batches, [6] walk
// cycles in total, [7] mode bits; trace kernel: [8] start / [9] end (s_memrealtime, 100 MHz),
// [10] work item, [11] chunk | chunks << 16 | last arriver << 32.
constexpr int kDiagBlocks = 65536;
constexpr int kDiagCols = 16;
__device__ unsigned long long g_srt_diag[kDiagBlocks][kDiagCols];
#define SRT_STAMP(v) const unsigned long long v = __builtin_amdgcn_s_memtime()
// Setup-kernel timelines (s_memrealtime, 100 MHz) of frame z = 0, thread 0 of each block:
// rows kDiagOrderRow + block (WorkOrderKernel), kDiagBinRow + block (PrepareBinKernel); column 0
// = block start, then one stamp per phase boundary (SRT_SETUP_MARK), column 15 = phases marked.
constexpr int kDiagOrderRow = 60000, kDiagBinRow = 61000;
#define SRT_SETUP_MARK(row, k)                                                                       \
    do {                                                                                             \
        if (threadIdx.x == 0 && blockIdx.z == 0 && (row) < kDiagBlocks) {                           \
            g_srt_diag[(row)][(k)] = __builtin_amdgcn_s_memrealtime();                               \
            g_srt_diag[(row)][15] = (k) + 1;                                                         \
        }                                                                                            \
    } while (0)
// Timing experiments of the diagnostic build (env SRT_EXP bits, the kernels' `exp` parameter): compiled
// out of the product, where every SRT_EXP_BIT is false.
#define SRT_EXP_BIT(p, bit) (((p).exp & (bit)) != 0u)
#else
#define SRT_STAMP(v)
#define SRT_SETUP_MARK(row, k)
#define SRT_EXP_BIT(p, bit) false
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
    const float4* __restrict__ shade;  // per triangle: (shading normal, |normal|), (albedo, 0) -- ShadeTableKernel
    const float2* __restrict__ offsets;
    float4* __restrict__ out;
    int* __restrict__ out_ids;  // non-null: store the hit id per pixel (-1 = miss) instead of RGBA
    unsigned char* __restrict__ out_packed;  // non-null: store packed ids (render.h PackedIds) instead
    int id_planes;             // packed ids: bit planes above the low 16 bits
    unsigned id_words;         // packed ids: 64-bit words per row and plane
    unsigned id_low_row_bytes; // packed ids: the row's u16 values (padded to 8 B), then its plane words
    unsigned id_row_bytes;     // packed ids: bytes per row
    unsigned id_tile_row_bytes;  // packed ids: bytes per tile row (its rows, then its tiles' offsets)
    int out_frame_rows;  // RGBA out is a whole frame: band row y stores at its frame row (render.h BandArgs)
    unsigned n_pad;   // records in the edge buffer (multiple of kPadTriangles)
    unsigned n;       // records in the scene
    int tiles_x;         // cull tiles per tile row of the band
    unsigned tiles;      // cull tiles of the band
    unsigned n_tiles; // tiles holding at least one real record (>= 1)
    int width;
    int row_count;
    int row_begin;
    int row_interleave;  // band = frame tile rows row_begin / kTileRows + k * row_interleave (1: contiguous rows)
    // Cull variant with bins (render.h CullBins); tile_info == null: no bins, every tile
    // computes its own ray box and streams every record.
    const TileInfo* __restrict__ tile_info;   // per tile: ray box, uniform offset (TileInfoKernel)
    const CullRecord* __restrict__ cull;      // cull records in spatial order (the lists hold positions)
    const unsigned* __restrict__ order;       // spatial-order position -> record id
    const float* __restrict__ svertices;      // vertices by spatial-order position (binned trace: records recomputed)
    const uint4* __restrict__ work;           // tile parts (2 x uint4 each), most work first (BuildWorkOrder)
    const unsigned* __restrict__ work_count;  // [0]: tile parts listed
    unsigned long long* __restrict__ split_keys;  // key slices of split parts: one per split slot, kBlockRows x 64 each
    unsigned* __restrict__ arrive;            // per split part (its first slot): chunks finished (self-resetting)
    const unsigned* __restrict__ bin_lists;   // per tile: candidate positions (PrepareBinKernel)
    const unsigned* __restrict__ bin_counts;  // per tile: list length; [tiles]: large-list length (this frame's)
    unsigned* __restrict__ bin_counts_next;   // the slot's other count buffer: reset by the trace for its next frame
    const unsigned* __restrict__ large_list;  // ids of records binned to every tile
    const unsigned* __restrict__ range_tag;   // = gen: some sample offset of this frame lies outside [0, 1]
    unsigned gen;                              // frame number of the scene (never 0)
    unsigned fused;                            // bins from the analytic tile bounds (BinParams::fused)
    unsigned plan_only;  // the work list is the slot's plan (no order launch for this frame): read the bins
    unsigned bin_capacity;
    unsigned exp;                                // diagnostic build: experiment bits (env SRT_EXP), 0 in the product
    float wf;
    float hf;
    float base[3];
    float du[3];
    float dv[3];
    float bg[3];
    float eye[3];  // ray origin (the 16-bit id decode recomputes candidate records)
};

// Frames of one batched launch: block (x, y, z) works on frame z. Up to kMaxBatch frames carry
// their parameters in the kernel-argument segment (FrameArgs); larger launches (up to
// kMaxTableFrames) read them from a device table the host uploads once per launch (FrameTable),
// through a constant-address-space pointer, so they compile to the same uniform scalar loads as
// kernel arguments (loads the compiler may treat as invariant and hoist).
template <class T>
using ConstantPtr = const __attribute__((address_space(4))) T*;
template <class T>
struct FrameArgs {
    T f[kMaxBatch];
    __device__ __forceinline__ const T& operator[](unsigned z) const { return f[z]; }
};
template <class T>
struct FrameTable {
    ConstantPtr<T> f;
    __device__ __forceinline__ const T& operator[](unsigned z) const { return *(const T*)(f + z); }
};
using TraceBatch = FrameArgs<TraceParams>;
using TraceTable = FrameTable<TraceParams>;

struct PrepareParams {
    const float* __restrict__ vertices;
    const unsigned* __restrict__ rank;  // record id -> position in the spatial order
    const unsigned* __restrict__ order; // position -> record id (the fused bin pass)
    const float* __restrict__ svertices;  // vertices by position (the fused bin pass)
    float4* __restrict__ edges;
    float4* __restrict__ screen_boxes;
    uint2* __restrict__ qboxes;
    CullRecord* __restrict__ cull;
    const float2* __restrict__ block_ext;  // render.h CullBins::block_ext (null: no block skip)
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
    const double dv[3] = {dBC, dCA, dAB};  // corner v's determinant: lines (v + 1) % 3, (v + 2) % 3
    for (int v = 0; v < 3; ++v) {
        const int i = (v + 1) % 3, j = (v + 2) % 3;  // corner opposite edge v: lines i and j
        // One division per corner: x, y and the pads multiply by 1 / d, which adds ~2 ulp (4e-16)
        // of relative error to x and y, far inside the 1e-12 pads (four divisions per corner
        // before). d is a nonzero difference of exact products of floats, so |d| >= 2^-298 and
        // 1 / d is finite; the guard keeps a NaN corner (0 x inf), which fmin / fmax would drop,
        // from ever shrinking the box.
        const double inv = 1.0 / dv[v], ainv = fabs(inv);
        if (!(ainv < 1e300)) {
            return unbounded;
        }
        const double tx1 = -k[i] * gy[j], tx2 = k[j] * gy[i];
        const double ty1 = -gx[i] * k[j], ty2 = gx[j] * k[i];
        const double x = (tx1 + tx2) * inv, y = (ty1 + ty2) * inv;
        const double px = 1e-12 * ((fabs(tx1) + fabs(tx2)) * ainv + fabs(x)) + 1e-300;
        const double py = 1e-12 * ((fabs(ty1) + fabs(ty2)) * ainv + fabs(y)) + 1e-300;
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

// Record of triangle `id` (real = a scene triangle, else padding): origin-relative edge normals
// nA = B x C, nB = C x A, nC = A x B (A, B, C = vertices - eye), signed volume vol = A . nA,
// orientation normalised so vol > 0, then each normal projected onto the affine ray frame:
// E(fx, fy) = n . (base + fx du + fy dv): c = (c0A, cxA, cyA, c0B, cxB, cyB, c0C, cxC, cyC).
// Disabled (padding, degenerate, plane through the eye): NaN record, empty screen box.
// v = the triangle's 9 vertex coordinates.
// The edge coefficients and vol alone (ComputeRecord without the screen box), under the frame
// (origin, base, du, dv); returns false for a disabled record (c, vol NaN). One definition for the
// record pass and the 16-bit id decode, so both see the same bits.
__device__ __forceinline__ bool ComputeEdges(const float* origin, const float* base, const float* du, const float* dv,
                                             const float* __restrict__ v, bool real, float c[9], float& vol) {
    const float qnan = __builtin_nanf("");
    bool disabled = !real;
    vol = qnan;
    if (!disabled) {
        const float ax = v[0] - origin[0], ay = v[1] - origin[1], az = v[2] - origin[2];
        const float bx = v[3] - origin[0], by = v[4] - origin[1], bz = v[5] - origin[2];
        const float cx = v[6] - origin[0], cy = v[7] - origin[1], cz = v[8] - origin[2];
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
                c[3 * e + 0] = Dot3(nx, ny, nz, base[0], base[1], base[2]);
                c[3 * e + 1] = Dot3(nx, ny, nz, du[0], du[1], du[2]);
                c[3 * e + 2] = Dot3(nx, ny, nz, dv[0], dv[1], dv[2]);
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
    return !disabled;
}

__device__ __forceinline__ void ComputeRecord(const PrepareParams& p, const float* __restrict__ v, bool real, float c[9],
                                              float& vol, float4& sb) {
    bool disabled = !ComputeEdges(p.origin, p.base, p.du, p.dv, v, real, c, vol);
    // Disabled records: an empty box (culled by every ray box the screen boxes apply to).
    sb = disabled ? make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff())
                  : make_float4(0.f, 0.f, 0.f, 0.f);
#ifdef SRT_DIAG
    disabled = disabled || SRT_EXP_BIT(p, 512u);  // timing experiment: 512 skips the screen box
#endif
    if (!disabled) {
        // The float solve with proven error bounds where it applies (screen_box.h: every record of
        // the soups), else the double one. (Measured: the double solve alone was ~3.8 us of a
        // single frame's 13 us record + bin launch -- a dependent chain of ~300 f64 instructions
        // at 1.5 waves per SIMD -- and ~0.6 us per frame of a P = 8 band rank's 5.7.)
        float fb[4];
        sb = ScreenBoxFast(c, kScreenBoxRange, fb) ? make_float4(fb[0], fb[1], fb[2], fb[3]) : ScreenBox(c);
    }
}

// ComputeRecord for the band record pass: the float solve's y half only, its x half left pending
// (`xpend`: finish it with ScreenBoxX(bs, sb.x, sb.y)) -- a record the band cannot see never needs
// it. Any other outcome (disabled, double solve, unbounded) is the whole box, as ComputeRecord's.
__device__ __forceinline__ void ComputeRecordY(const PrepareParams& p, const float* __restrict__ v, bool real,
                                               float c[9], float& vol, float4& sb, BoxSolve& bs, bool& xpend) {
    xpend = false;
    const bool disabled = !ComputeEdges(p.origin, p.base, p.du, p.dv, v, real, c, vol);
    sb = make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff());
    if (disabled) {
        return;
    }
    ScreenBoxSetup(c, kScreenBoxRange, bs);
    if (!bs.ok) {
        sb = ScreenBox(c);
    } else if (!bs.spans) {
        sb = make_float4(-__builtin_inff(), __builtin_inff(), -__builtin_inff(), __builtin_inff());
    } else {
        ScreenBoxY(bs, sb.z, sb.w);
        xpend = true;
    }
}

// Stored as (hi, -lo) pairs so the cull test is one saturating packed add per axis.
__device__ __forceinline__ uint2 QuantizeBox(const float4& sb) {
    return make_uint2(PackI16(QuantHi(sb.y), -QuantLo(sb.x)), PackI16(QuantHi(sb.w), -QuantLo(sb.z)));
}

// Shading normal of the triangle with vertex coordinates v[0..9): the exact expressions the
// shading epilogue used to evaluate per hit.
__device__ __forceinline__ float4 ShadingNormal(const float* __restrict__ v) {
    const float e1x = v[3] - v[0], e1y = v[4] - v[1], e1z = v[5] - v[2];
    const float e2x = v[6] - v[0], e2y = v[7] - v[1], e2z = v[8] - v[2];
    float nx, ny, nz;
    Cross3(e1x, e1y, e1z, e2x, e2y, e2z, nx, ny, nz);
    return make_float4(nx, ny, nz, sqrtf(Dot3(nx, ny, nz, nx, ny, nz)));
}

// Shading table of a scene (once, at load): triangle i -> (ShadingNormal, (albedo, 0)).
__global__ __launch_bounds__(256) void ShadeTableKernel(const float* __restrict__ vertices,
                                                        const float* __restrict__ albedo, unsigned n,
                                                        float4* __restrict__ table) {
    const unsigned i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        table[2ull * i] = ShadingNormal(vertices + 9ull * i);
        table[2ull * i + 1] = make_float4(albedo[3ull * i], albedo[3ull * i + 1], albedo[3ull * i + 2], 0.f);
    }
}

// The full record pass (every variant but the binned cull path, which fuses it into its bin
// kernel): one thread per record id i, writing the tile-planar edge record, the screen box, and
// at the record's spatial position (rank[i]; padding ids are their own position) its quantized
// box and cull record; the shading normal by id.
__device__ __forceinline__ void PrepareRecord(const PrepareParams& p, unsigned i) {
    if (i >= p.n_pad) {
        return;
    }
    float4* tile = p.edges + static_cast<size_t>(i / kTileTriangles) * kTileFloat4;
    const unsigned j = i % kTileTriangles;
    float* p2 = reinterpret_cast<float*>(tile + 2 * kTileTriangles);
    float* p3 = p2 + kTileTriangles;
    const bool real = i < p.n;
    float c[9], vol;
    float4 sb;
    ComputeRecord(p, p.vertices + 9ull * i, real, c, vol, sb);
    tile[j] = make_float4(c[0], c[1], c[2], c[3]);
    tile[kTileTriangles + j] = make_float4(c[4], c[5], c[6], c[7]);
    p2[j] = c[8];
    p3[j] = vol;
    p.screen_boxes[i] = sb;
    const unsigned pos = real ? p.rank[i] : i;
    p.qboxes[pos] = QuantizeBox(sb);
    CullRecord r;
    r.a = make_float4(c[0], c[1], c[2], c[3]);
    r.b = make_float4(c[4], c[5], c[6], c[7]);
    r.x = make_float4(c[8], vol, __uint_as_float(i), 0.f);
    r.sb = sb;
    p.cull[pos] = r;
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
// Frame row of band-local row `local`: the band holds frame tile rows row_begin / kCullTileRows
// + k * interleave, k = 0, 1, ... (interleave 1: the contiguous rows row_begin + local).
// (interleave: a plain interleave, or a RowPattern taking 2^g consecutive tile rows of every
// interleave: render.h BandFrameRow; a shift and a mask, no branch.)
__device__ __forceinline__ int FrameRow(int row_begin, int interleave, int local) {
    const int lt = local / kCullTileRows, g = interleave >> 16;
    return row_begin + ((lt >> g) * (interleave & 0xFFFF) + (lt & ((1 << g) - 1))) * kCullTileRows +
           local % kCullTileRows;
}

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
        s.fy[r] = (static_cast<float>(FrameRow(p.row_begin, p.row_interleave, yc)) + o.y) / p.hf;
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

// Shade: rgb = albedo * |cos(N, d)| for a hit, background for a miss; alpha carries
// float(tri_id) (exact for ids < 2^24), -1 for a miss.
// The shading of a hit from its triangle's shading record (nr, a) -- built once at scene load from
// its vertices and albedo (static scene data, like the vertices themselves: 32 B, one line, instead of
// 36 B of vertices, 12 B of albedo and a cross product and square root per pixel); the same
// expressions, so the same bits. A miss (id < 0): the background.
__device__ __forceinline__ float4 ShadeRecord(const TraceParams& p, float fx, float fy, int id, const float4& nr,
                                              const float4& a) {
    if (id < 0) {
        return make_float4(p.bg[0], p.bg[1], p.bg[2], -1.f);
    }
    const float dx = fmaf(fy, p.dv[0], fmaf(fx, p.du[0], p.base[0]));
    const float dy = fmaf(fy, p.dv[1], fmaf(fx, p.du[1], p.base[1]));
    const float dz = fmaf(fy, p.dv[2], fmaf(fx, p.du[2], p.base[2]));
    const float nd = Dot3(nr.x, nr.y, nr.z, dx, dy, dz);
    const float dd = Dot3(dx, dy, dz, dx, dy, dz);
    const float cosv = fminf(fabsf(nd) / (nr.w * sqrtf(dd)), 1.f);
    return make_float4(a.x * cosv, a.y * cosv, a.z * cosv, static_cast<float>(id));
}
__device__ __forceinline__ float4 ShadePixel(const TraceParams& p, float fx, float fy, int id) {
    if (id < 0) {
        return ShadeRecord(p, fx, fy, id, float4{}, float4{});
    }
    const float4* sr = p.shade + 2ull * static_cast<unsigned>(id);
    return ShadeRecord(p, fx, fy, id, sr[0], sr[1]);
}

// Store one pixel of the band: its shaded RGBA (one float4, 1 KiB contiguous per wave
// instruction), or only its hit id (out_ids: deferred shading by ShadeIdsKernel, bit-identical).
// Nontemporal (`global_store ... nt`): the frame never reads its framebuffer back, and streaming
// it past the L2 keeps the cull records, lists and tables resident (+7.8 % at C3).
typedef float F4 __attribute__((ext_vector_type(4)));
// A nontemporal float4 store the compiler cannot merge: after ShadeIdsKernel's grid was compacted
// (its store no longer behind a row test), clang sank the two stores of ShadeRecord's hit / miss
// paths into one and dropped `nt` on the way (97 -> 112 us per 8-frame launch of a P = 8
// compositor; a branch-free ShadeRecord kept `nt` but shaded every miss: 104 us).
__device__ __forceinline__ void StoreNontemporal(F4* at, F4 v) {
    asm volatile("global_store_dwordx4 %0, %1, off nt" ::"v"(at), "v"(v) : "memory");
}
__device__ __forceinline__ void StoreRgba(const TraceParams& p, int x, int y, const float4& v) {
    const size_t rgba_at = p.out_frame_rows != 0
                               ? static_cast<size_t>(FrameRow(p.row_begin, p.row_interleave, y)) * p.width + x
                               : static_cast<size_t>(y) * p.width + x;
    __builtin_nontemporal_store(F4{v.x, v.y, v.z, v.w}, reinterpret_cast<F4*>(p.out + rgba_at));
}
__device__ __forceinline__ void StorePixel(const TraceParams& p, int x, int y, float fx, float fy, int id) {
    if (p.out_ids != nullptr) {
        __builtin_nontemporal_store(id, p.out_ids + static_cast<size_t>(y) * p.width + x);
    } else {
        StoreRgba(p, x, y, ShadePixel(p, fx, fy, id));
    }
}

// Packed ids (render.h PackedIds) of one band row segment: the wave's 64 lanes are the 64 columns
// x = tx * 64 + lane of band row y (wave-uniform; called by every lane of the wave). The low 16 bits
// go to the u16 plane; bit 16 + j of the 64 codes is one ballot, stored by lane 0 as plane j's word.
// Band row y of a packed band frame, and the offset entry of tile tx of band tile row y / kCullTileRows
// (render.h PackedIds).
template <class Byte>
__device__ __forceinline__ Byte* PackedRow(Byte* frame, const TraceParams& p, int y) {
    return frame + static_cast<size_t>(y / kCullTileRows) * p.id_tile_row_bytes +
           static_cast<size_t>(y % kCullTileRows) * p.id_row_bytes;
}
template <class Byte>
__device__ __forceinline__ Byte* PackedTileOffset(Byte* frame, const TraceParams& p, int y, int tx) {
    return frame + static_cast<size_t>(y / kCullTileRows) * p.id_tile_row_bytes +
           static_cast<size_t>(kCullTileRows) * p.id_row_bytes + static_cast<size_t>(tx) * sizeof(float2);
}

__device__ __forceinline__ void StorePackedIds(const TraceParams& p, int tx, int x, int y, int id) {
    const bool valid = x < p.width;
    const unsigned code = id < 0 ? 0xFFFFFFFFu : static_cast<unsigned>(id);
    unsigned char* row = PackedRow(p.out_packed, p, y);
    if (valid) {
        __builtin_nontemporal_store(static_cast<unsigned short>(code & 0xFFFFu), reinterpret_cast<unsigned short*>(row) + x);
    }
    unsigned long long* words = reinterpret_cast<unsigned long long*>(row + p.id_low_row_bytes);
    for (int j = 0; j < p.id_planes; ++j) {
        const unsigned long long m = __ballot(valid && ((code >> (16 + j)) & 1u) != 0u);
        if ((threadIdx.x & (kWave - 1)) == 0) {
            __builtin_nontemporal_store(m, words + static_cast<size_t>(j) * p.id_words + tx);
        }
    }
}

// Shade + store the lane's R rays.
template <int R>
__device__ __forceinline__ void ShadeAndStore(const TraceParams& p, int x, int y0, const Rays<R>& s) {
    if (x >= p.width) {
        return;
    }
#pragma unroll
    for (int r = 0; r < R; ++r) {
        const int y = y0 + r;
        if (y < p.row_count) {
            StorePixel(p, x, y, s.fx[r], s.fy[r], s.bi[r]);
        }
    }
}

// Deferred shading: one thread per pixel of a band, from its hit id and sample offset, with
// GenerateRays' position expressions and ShadePixel: the frame equals the fused trace + shade
// bit for bit. blockIdx.y = frame g of a batch whose ids arrive band-major, as a gather of
// `frames` frames of row bands leaves them: ids[band][g][band_rows][width] (one frame and one
// band of row_count rows: the plain (row_count, width) layout); out[g][row_count][width]. With
// `interleaved` bands the bands took the frame's tile rows round-robin: row y is row
// (t / bands) * kCullTileRows + y % kCullTileRows of band t % bands, t = y / kCullTileRows.
// Grid (ceil(W / kShadeThreads), ceil(row_count / kShadeRows), frames): block (bx, by, g) shades
// kShadeThreads columns x kShadeRows rows of frame g, a thread one column of kShadeRows rows with all
// their id and offset loads in flight together (no per-pixel division for x and y: the former 1-D
// grid's 64-bit i % W and i / W were most of the kernel's instructions).
#ifndef SRT_SHADE_THREADS
#define SRT_SHADE_THREADS 128
#endif
constexpr int kShadeThreads = SRT_SHADE_THREADS;
#ifndef SRT_SHADE_ROWS
// Rows per thread. Round 5, with every row's loads issued before any is used (the tile offsets pinned
// there, exact float row division): 1 / 2 / 4 rows 690 / 646 / 582 us per 128-frame launch of a P = 2
// compositor, 263 / 260 / 248 us per 32-frame launch at P = 8 (profiles/r05/shade_ab/rows.txt). (Before,
// clang serialised the rows' loads behind per-row branches: 2 rows measured slower than 1.)
#define SRT_SHADE_ROWS 4
#endif
constexpr int kShadeRows = SRT_SHADE_ROWS;

// (t, id) packed so that unsigned order is lexicographic order: t >= 0 here (vol > 0,
// det > 0), so its bit pattern orders like the value.
__device__ __forceinline__ unsigned long long HitKey(float t, int id) {
    return (static_cast<unsigned long long>(__float_as_uint(t)) << 32) | static_cast<unsigned>(id);
}

// Quotient of small unsigned integers, exact for y < 2^21 and any d >= 1: |fl(y + 1/2) * rcp(d) - (y +
// 1/2) / d| <= (y + 1/2) / d * 1.5 * 2^-23 (v_rcp_f32 within 1 ulp, one rounding of the product), below
// the 1 / (2 d) by which (y + 1/2) / d stays from an integer. The shading kernel's row mapping divides
// wave-uniform values, which clang expanded into ~25 scalar instructions each (117 SALU per wave, 62 % of
// the CU's scalar issue at a P = 8 compositor; PMC, profiles/r05/shade_pmc/).
__device__ __forceinline__ unsigned UDivSmall(unsigned y, unsigned d) {
    if (y >= (1u << 21)) {  // (frames of over 2M rows: the integer division)
        return y / d;
    }
    return static_cast<unsigned>((static_cast<float>(y) + 0.5f) * __builtin_amdgcn_rcpf(static_cast<float>(d)));
}
// The frame row of the j-th row a shade call stores: the rows of bands [0, own) and of band `skip`
// (~0u: none) left out. Interleaved (m = interleaved): band b is tile rows b, b + m, ... of 16 rows;
// else band b is rows [b * band_rows, (b + 1) * band_rows), or, with first_rows > 0, band 0 is rows
// [0, first_rows) and band b >= 1 rows [first_rows + (b - 1) * band_rows, ...). Past the last stored row the result is
// past the frame only if the caller's grid (ShadeRowsLaunched) stops at the frame's rows.
__device__ __forceinline__ unsigned ShadeRowOf(unsigned j, unsigned band_rows, unsigned interleaved, unsigned skip,
                                               unsigned own, unsigned first_rows) {
    const bool skips = skip != ~0u && skip >= own;
    if (interleaved != 0u) {
        const unsigned stored = interleaved - own - (skips && skip < interleaved ? 1u : 0u);
        const unsigned tr = j / kCullTileRows;
        const unsigned q = UDivSmall(tr, stored);
        unsigned band = own + (tr - q * stored);
        band += skips && band >= skip ? 1u : 0u;
        return (q * interleaved + band) * kCullTileRows + j % kCullTileRows;
    }
    // contiguous: band b starts at row b == 0 ? 0 : F + (b - 1) S (F = first_rows, or S = band_rows)
    const unsigned long long F = first_rows != 0u ? first_rows : band_rows, S = band_rows;
    const auto start = [&](unsigned b) { return b == 0u ? 0ull : F + (b - 1ull) * S; };
    unsigned long long y = start(own) + j;
    y += skips && y >= start(skip) ? (skip == 0u ? F : S) : 0ull;
    return y > 0x7FFFFFFFull ? 0x7FFFFFFFu : static_cast<unsigned>(y);
}

// PACKED: the ids arrive as packed band frames (render.h PackedIds, frame_bytes each, the same
// band-major order): a pixel's code is its u16 plus p.id_planes bits from the bit planes.
template <bool PACKED, int PLANES>
__global__ __launch_bounds__(kShadeThreads) void ShadeIdsKernel(TraceParams p, const void* __restrict__ ids_v,
                                                                unsigned band_rows, unsigned frames,
                                                                unsigned interleaved, size_t offsets_stride,
                                                                unsigned skip_band, unsigned own_bands,
                                                                size_t frame_bytes, unsigned first_rows) {
    static_assert(kShadeThreads % kWave == 0, "a wave's lanes are one 64-column tile column");
    const int* __restrict__ ids = static_cast<const int*>(ids_v);
    const unsigned char* __restrict__ packed = static_cast<const unsigned char*>(ids_v);
    const int x = static_cast<int>(blockIdx.x * kShadeThreads + threadIdx.x);
    if (x >= p.width) {
        return;
    }
    // The grid covers only the rows this call stores (ShadeRowsLaunched): blockIdx.y counts them,
    // the bands [0, own_bands) and skip_band left out, and ShadeRowOf maps the count to its frame row.
    // (A grid over every row, whose own-band threads loaded and stored nothing, cost a compositor of
    // the share exchange -- a fifth of its rows shaded -- 7.3 us per frame, 2.6 us compacted.)
    const unsigned j0 = blockIdx.y * kShadeRows;
    const int y0 = static_cast<int>(ShadeRowOf(j0, band_rows, interleaved, skip_band, own_bands, first_rows));
    if (y0 >= p.row_count) {
        return;
    }
    const unsigned g = blockIdx.z;
    const size_t pixels = static_cast<size_t>(p.width) * p.row_count;
    // Three phases with no control flow between the loads of different rows, so every row's loads are
    // in flight together: (1) every row's id (packed: its u16, bit-plane words and tile offset --
    // wave-uniform addresses), (2) every hit's sample offset (irregular tiles) and every row's shading
    // record, (3) shade and store. (The per-row form waited on each row's planes and each hit's record
    // in turn: 3 round trips per row.) A row past the frame loads from a valid one and is not stored.
    // Interleaved bands: the thread's rows lie in one tile row (kShadeRows divides it), so in one
    // band (the divisions once per thread, not per row); contiguous bands map row by row (a thread's
    // rows may straddle skip_band).
    static_assert(kCullTileRows % kShadeRows == 0, "a thread's rows share a tile row");
    const unsigned t0 = static_cast<unsigned>(y0) / kCullTileRows;
    const unsigned tq = interleaved != 0u ? UDivSmall(t0, interleaved) : 0u;
    const unsigned band0 = interleaved != 0u ? t0 - tq * interleaved : 0u;
    const unsigned local0 = interleaved != 0u ? tq * kCullTileRows + static_cast<unsigned>(y0) % kCullTileRows : 0u;
    const int tcol = __builtin_amdgcn_readfirstlane(x >> 6);  // the wave's tile column
    unsigned code[kShadeRows];
    float2 tile_o[kShadeRows];  // packed ids: the row's tile offset (NaN: every pixel reads its own)
    int yr[kShadeRows];         // frame rows (>= row_count: past the frame, not stored)
    unsigned long long plane[kShadeRows][PLANES > 0 ? PLANES : 1];  // packed ids: the rows' bit-plane words
    // (The bands [0, own_bands) hold no ids in the buffer, which starts at band own_bands: the
    // compositor traced them as RGBA already.)
#pragma unroll
    for (int r = 0; r < kShadeRows; ++r) {
        yr[r] = interleaved != 0u || r == 0
                    ? y0 + r
                    : static_cast<int>(ShadeRowOf(j0 + r, band_rows, interleaved, skip_band, own_bands, first_rows));
        const bool past = yr[r] >= p.row_count;
        const unsigned y = static_cast<unsigned>(past ? y0 : yr[r]);
        unsigned band, local;
        if (interleaved != 0u) {
            band = band0;
            local = local0 + (y - static_cast<unsigned>(y0));
        } else if (first_rows != 0u) {
            band = y < first_rows ? 0u : 1u + UDivSmall(y - first_rows, band_rows);
            local = band == 0u ? y : y - first_rows - (band - 1u) * band_rows;
        } else {
            band = UDivSmall(y, band_rows);
            local = y - band * band_rows;
        }
        const unsigned slot = band - own_bands;
        if constexpr (PACKED) {
            const unsigned char* frame = packed + (static_cast<size_t>(slot) * frames + g) * frame_bytes;
            const unsigned char* row = PackedRow(frame, p, static_cast<int>(local));
            code[r] = reinterpret_cast<const unsigned short*>(row)[x];
            const unsigned long long* bits = reinterpret_cast<const unsigned long long*>(row + p.id_low_row_bytes);
#pragma unroll
            for (int j = 0; j < PLANES; ++j) {
                plane[r][j] = bits[static_cast<size_t>(j) * p.id_words + tcol];
            }
            tile_o[r] = *reinterpret_cast<const float2*>(PackedTileOffset(frame, p, static_cast<int>(local), tcol));
        } else {
            const size_t at = ((static_cast<size_t>(slot) * frames + g) * band_rows + local) * p.width + x;
            code[r] = static_cast<unsigned>(__builtin_nontemporal_load(ids + at));
            tile_o[r] = make_float2(__builtin_nanf(""), __builtin_nanf(""));
        }
    }
    // Every row's loads are issued above before any is used (the codes are assembled here). Only a hit
    // uses the tile offset, so clang sank its (scalar) load into the hit branch, behind the u16 load's
    // wait: a third round trip in the chain (u16 -> tile offset -> shading record). Pinned here, it is
    // in flight with the u16s and the bit-plane words.
    if constexpr (PACKED) {
#pragma unroll
        for (int r = 0; r < kShadeRows; ++r) {
#pragma unroll
            for (int j = 0; j < PLANES; ++j) {
                code[r] |= static_cast<unsigned>((plane[r][j] >> (x & 63)) & 1ull) << (16 + j);
            }
            asm volatile("" ::"s"(tile_o[r].x), "s"(tile_o[r].y));
        }
    }
    // Only a hit needs its ray: a miss shades to the background whatever its sample offset (a miss is
    // -1, the packed miss code -- all ones -- or any id outside the scene). A hit in a regular tile
    // takes the tile's offset (the trace computed its ray from the same one, bit for bit); in other
    // rows every lane reads its own (a wave-uniform branch: the tile offset is one scalar per wave and
    // row, so no lane mask splits the row's loads from the others'). Every row's shading record is
    // loaded (a miss's: triangle 0's, unused).
    int hit[kShadeRows];
    float2 o[kShadeRows];
    float4 nr[kShadeRows], al[kShadeRows];
#pragma unroll
    for (int r = 0; r < kShadeRows; ++r) {
        const int y = yr[r] < p.row_count ? yr[r] : y0;
        hit[r] = code[r] < p.n ? static_cast<int>(code[r]) : -1;
        const bool regular = PACKED && tile_o[r].x == tile_o[r].x;
        o[r] = tile_o[r];
        if (!regular) {
            o[r] = p.offsets[static_cast<size_t>(y) * p.width + x + g * offsets_stride];  // frame g's (stride 0: shared)
        }
        const float4* sr = p.shade + 2ull * static_cast<unsigned>(max(hit[r], 0));
        nr[r] = sr[0];
        al[r] = sr[1];
    }
#pragma unroll
    for (int r = 0; r < kShadeRows; ++r) {
        const int y = yr[r];
        if (y < p.row_count) {
            const float fx = (static_cast<float>(x) + o[r].x) / p.wf;
            const float fy = (static_cast<float>(FrameRow(p.row_begin, p.row_interleave, y)) + o[r].y) / p.hf;
            const float4 v = ShadeRecord(p, fx, fy, hit[r], nr[r], al[r]);
            StoreNontemporal(reinterpret_cast<F4*>(p.out + g * pixels + static_cast<size_t>(y) * p.width + x),
                             F4{v.x, v.y, v.z, v.w});
        }
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

// Cull tile = 64 columns x kTileRows rows of rays (the bins); trace block = one part of it,
// 64 columns x kBlockRows rows: kCullWaves waves, each 64 columns x kCullR rows (lane =
// column).
constexpr int kTileRows = kCullTileRows;
#ifndef SRT_BLOCK_ROWS
#define SRT_BLOCK_ROWS 16
#endif
constexpr int kBlockRows = SRT_BLOCK_ROWS;
constexpr int kParts = kTileRows / kBlockRows;
#ifndef SRT_CULL_WAVES
#define SRT_CULL_WAVES 4
#endif
constexpr int kCullWaves = SRT_CULL_WAVES;
constexpr int kCullThreads = kWave * kCullWaves;
constexpr int kCullR = kBlockRows / kCullWaves;  // rays per lane
#ifndef SRT_PACKET_BATCH
#define SRT_PACKET_BATCH 128
#endif
#ifndef SRT_LANE_PIXELS
#define SRT_LANE_PIXELS 2  // packet walk: consecutive range pixels per lane (one record read for them)
#endif
#ifndef SRT_PACKET_ILP
#define SRT_PACKET_ILP 1  // packet walk: packets evaluated together per wave (independent chains)
#endif
constexpr int kPacketBatch = SRT_PACKET_BATCH;  // candidates gathered per packet-walk batch
constexpr unsigned kLanePixels = SRT_LANE_PIXELS;
constexpr int kSlices = (kPacketBatch + kCullThreads - 1) / kCullThreads;  // batch entries per thread
constexpr int kStreamStep = kCullThreads;        // FULL stream: records per block per step
static_assert((kPacketBatch % kCullThreads == 0 || kCullThreads % kPacketBatch == 0) && kPacketBatch <= 256,
              "whole slices (or a part of the threads); packet word: survivor slot < 256");
static_assert(kBlockRows <= 16 && kBlockRows % kCullWaves == 0, "packet word: rows < 16");
static_assert(kPadTriangles % kStreamStep == 0, "a stream step must cover whole pad units");

#ifndef SRT_WINDOW_PACKETS
#define SRT_WINDOW_PACKETS 128
#endif
constexpr int kWindowPackets = SRT_WINDOW_PACKETS;  // packet walk: packets per window of the pixel stream
constexpr unsigned kWindowPixels = kWindowPackets * kWave;
static_assert(kWindowPackets == 2 * kWave, "window prefix: two packets per lane");

// Batch entry of thread tid's slice e (kPacketBatch < kCullThreads: the first threads only).
__device__ __forceinline__ bool InBatch(int e, int tid) { return e * kCullThreads + tid < kPacketBatch; }

struct CullShared {
    union {
        struct {
            float4 sv0[kPacketBatch];  // compacted survivors: plane 0 (sv0, sv1 adjacent: PacketTables scratch)
            float4 sv1[kPacketBatch];  //                      plane 1
            float4 sv2[kPacketBatch];  //                      (cyC, vol, id, 1 / nc)
        };
        unsigned ids[kPacketBatch + kStreamStep];  // FULL stream: surviving record ids (read into
                                                   // registers before a batch writes the planes)
    };
    uint2 aux[kPacketBatch + 1];  // per survivor: (exclusive pixel prefix, range base pixel byte offset | nc << 16);
                                  // aux[S].x = pixels of the batch
    unsigned wave_n[kSlices * kCullWaves];   // survivors per (slice, wave)
    unsigned wave_pk[kSlices * kCullWaves];  // pixels per (slice, wave)
    uint2 pk[2][kWindowPackets];  // window packet k: last-pixel bits (lo, hi); two buffers, alternate batches
    float2 fxy[kBlockRows][kWave];  // ray position (fx, fy) of every pixel of the block (512-B rows:
                                    // rows padded by 8 or 16 B to skew the banks measured 3-6 % slower)
    float clo[kWave], chi[kWave];    // monotone column bounds of fx (suffix min, prefix max)
    float rlo[kBlockRows], rhi[kBlockRows];  // monotone row bounds of fy
    unsigned counts[2][kCullWaves];            // FULL stream: survivors per wave and step
    Box wave_box[kCullWaves];
    unsigned last;  // split work item: this block arrived last
    unsigned long long keys[kBlockRows][kWave];  // per-pixel lexicographic (t, id) keys
};
static_assert(sizeof(float2) * kWave * kCullWaves <= sizeof(float4) * 2 * kPacketBatch, "PacketTables scratch");
static_assert((kPacketBatch + kStreamStep) * 4 <= sizeof(float4) * 3 * kPacketBatch, "stream ids alias the planes");
constexpr int kFlushBatches = (kPacketBatch + kStreamStep - 1 + kPacketBatch - 1) / kPacketBatch;  // per flush


// Candidate source of a block: LIST = positions [begin, end) of the tile's virtual list (its
// bin list, then the large list of records binned to every tile); FULL = every record.
struct CullSource {
    const unsigned* list;   // LIST: the tile's list (virtual positions < count1)
    const unsigned* list2;  // LIST: large list (virtual position v >= count1: list2[v - count1])
    unsigned count1;
    unsigned begin;
    unsigned end;
    bool full;
};

// ---------------------------------------------------------------------------------------
// Packet walk. The block's 64 x 16 ray positions sit in an LDS table; per column the
// smallest and largest fx over the block's rows, per row the smallest and largest fy over
// its columns, made monotone (lo' = suffix minimum, hi' = prefix maximum; a uniform-offset
// tile's tables are single values, already monotone). Per batch of up to kPacketBatch
// candidates:
//   filter:  one thread per candidate keeps it if it passes the block-box tests
//            (ScreenBoxOverlaps, BoxMayHit) and finds the columns whose fx interval can meet
//            its screen box (hi'[c] >= xlo, lo'[c] <= xhi: searches in the monotone tables),
//            and likewise the rows. A pixel outside those ranges has fx or fy outside the
//            screen box, so it cannot pass the exact test (screen-box guarantee): skipping it
//            is exact. (A block box outside the screen-box range: no screen-box tests, the
//            whole block is the range.);
//   compact: survivors are compacted block-wide in any order, with an exclusive prefix of
//            their pixel counts: the batch's pixel stream, every range row-major, back to back;
//   walk:    the stream is cut into packets of 64 consecutive pixels, which may span several
//            survivors (dense: round 1 padded every range to whole packets, 56 % of the lanes
//            busy at C3); wave w takes the packets [w P / W, (w + 1) P / W) of a window's P, two
//            per iteration (independent dependency chains for the scheduler): each lane finds
//            its survivor from the window's range-end bitmap, reads its pixel's (fx, fy), tests
//            it exactly and merges a hit into the pixel's key with an LDS atomic min.
// Same exact test and lexicographic (t, id) result as ExactTestAnyOrder.
// ---------------------------------------------------------------------------------------
struct PacketHit {
    unsigned long long key;
    bool hit;
};

struct PacketPixel {
    unsigned pixb;  // byte offset of the pixel in an 8-B-per-pixel block table (keys, positions)
    bool in;        // a pixel of the stream (lanes past its end address pixel 0)
};

__device__ __forceinline__ PacketHit EvalPacket(const float4& a, const float4& b, const float4& x, float2 f,
                                                bool in) {
    const float eA = fmaf(f.y, a.z, fmaf(f.x, a.y, a.x));
    const float eB = fmaf(f.y, b.y, fmaf(f.x, b.x, a.w));
    const float eC = fmaf(f.y, x.x, fmaf(f.x, b.w, b.z));
    const float det = (eA + eB) + eC;
    const float t = x.y / det;
    PacketHit h;
    h.hit = static_cast<bool>(in & (fminf(fminf(eA, eB), eC) >= 0.f) & (det > 0.f) & (t < __builtin_inff()));
    h.key = HitKey(t, __float_as_int(x.z));
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

// Inclusive scans over the 64 lanes of a wave: prefix maximum (up) / suffix minimum (down).
__device__ __forceinline__ float WavePrefixMax(float v, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const float u = __shfl_up(v, o);
        v = lane >= o ? fmaxf(v, u) : v;
    }
    return v;
}
__device__ __forceinline__ float WaveSuffixMin(float v, int lane) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        const float u = __shfl_down(v, o);
        v = lane + o < kWave ? fminf(v, u) : v;
    }
    return v;
}
__device__ __forceinline__ float WaveMin(float v) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        v = fminf(v, __shfl_xor(v, o));
    }
    return v;
}
__device__ __forceinline__ float WaveMax(float v) {
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        v = fmaxf(v, __shfl_xor(v, o));
    }
    return v;
}

// The block's position tables (see the section comment) from the lane's rays. `regular`:
// every ray of the block has the same sample offset, so fx_lane (column `lane`) and fy_lane
// (row `lane` < kBlockRows) already are the monotone tables. Ends with a barrier.
__device__ __forceinline__ void PacketTables(CullShared& sh, const Rays<kCullR>& s, bool regular, float fx_lane,
                                             float fy_lane, int nc, int nr) {
    constexpr int R = kCullR;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
#pragma unroll
    for (int r = 0; r < R; ++r) {
        sh.fxy[wave * R + r][lane] = make_float2(s.fx[r], s.fy[r]);
    }
    if (regular) {
        if (tid < kWave) {
            sh.clo[tid] = fx_lane;
            sh.chi[tid] = fx_lane;
        }
        if (tid < kBlockRows) {
            sh.rlo[tid] = fy_lane;
            sh.rhi[tid] = fy_lane;
        }
        __syncthreads();
        return;
    }
    // Per column: min / max of fx over this wave's rows (scratch in the survivor planes, which
    // the first batch writes only after later barriers); per row: over the valid columns.
    float2* part = reinterpret_cast<float2*>(sh.sv0);
    float lo = __builtin_inff(), hi = -__builtin_inff();
#pragma unroll
    for (int r = 0; r < R; ++r) {
        lo = fminf(lo, s.fx[r]);
        hi = fmaxf(hi, s.fx[r]);
        const float fy = lane < nc ? s.fy[r] : __builtin_nanf("");  // NaN drops out of min / max
        const float ylo = WaveMin(fy), yhi = WaveMax(fy);
        if (lane == 0) {
            sh.rlo[wave * R + r] = ylo;
            sh.rhi[wave * R + r] = yhi;
        }
    }
    part[wave * kWave + lane] = make_float2(lo, hi);
    __syncthreads();
    if (wave == 0) {
        float clo = __builtin_inff(), chi = -__builtin_inff();
#pragma unroll
        for (int w = 0; w < kCullWaves; ++w) {
            const float2 v = part[w * kWave + lane];
            clo = fminf(clo, v.x);
            chi = fmaxf(chi, v.y);
        }
        // Columns past the frame edge do not constrain the valid ones (searches stop at nc).
        sh.clo[lane] = WaveSuffixMin(lane < nc ? clo : __builtin_inff(), lane);
        sh.chi[lane] = WavePrefixMax(chi, lane);
    } else if (wave == 1) {
        const float rl = lane < nr ? sh.rlo[min(lane, kBlockRows - 1)] : __builtin_inff();
        const float rh = lane < kBlockRows ? sh.rhi[lane] : -__builtin_inff();
        const float rlo = WaveSuffixMin(rl, lane), rhi = WavePrefixMax(rh, lane);
        if (lane < kBlockRows) {
            sh.rlo[lane] = rlo;
            sh.rhi[lane] = rhi;
        }
    }
    __syncthreads();
}

// Per-block constants of the packet walk: valid columns / rows and the linear models of the
// monotone tables for the range guesses; use_sb = the block box is inside the screen-box range.
struct PacketFrame {
    int nc, nr;
    bool use_sb;
    float fx_first, fx_scale, fy_first, fy_scale;
};
__device__ __forceinline__ PacketFrame MakePacketFrame(const CullShared& sh, int nc, int nr, bool use_sb) {
    PacketFrame f;
    f.nc = nc;
    f.nr = nr;
    f.use_sb = use_sb;
    f.fx_first = sh.clo[0];
    f.fy_first = sh.rlo[0];
    const float fx_last = sh.chi[nc - 1], fy_last = sh.rhi[nr - 1];
    f.fx_scale = nc > 1 && fx_last > f.fx_first ? static_cast<float>(nc - 1) / (fx_last - f.fx_first) : 0.f;
    f.fy_scale = nr > 1 && fy_last > f.fy_first ? static_cast<float>(nr - 1) / (fy_last - f.fy_first) : 0.f;
    return f;
}

// One packet-walk batch: candidate e * kCullThreads + tid is cr[e] when valid[e]. Filter,
// compaction and the walk into sh.keys; `prefetch()` runs between the compaction and the walk
// (the next batch's loads then hide behind the walk). Starts and ends with block-uniform
// control flow. Two barriers for a batch of <= kWindowPixels pixels, none at the end: the next
// batch's first barrier separates this walk from its plane writes, the range-end bitmap
// alternates between two buffers (`buf` = batch parity; this batch clears the other one), and
// the caller puts a barrier between the last batch and its reads of sh.keys.
template <class F>
__device__ __forceinline__ void PacketBatch(CullShared& sh, const Box& bb, const PacketFrame& pf,
                                            const CullRecord (&cr)[kSlices], const bool (&valid)[kSlices],
                                            unsigned buf, F&& prefetch) {
    constexpr int W = kCullWaves;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    const unsigned long long lt_mask = (1ull << lane) - 1ull;
    uint2* pkb = sh.pk[buf];
    bool pass[kSlices];
    unsigned bits[kSlices], npk[kSlices];  // bits: range base pixel byte offset | range width << 16
#pragma unroll
    for (int e = 0; e < kSlices; ++e) {
        bits[e] = 0u;
        npk[e] = 0u;
        const float4 sb = cr[e].sb;
        const Record r{cr[e].a.x, cr[e].a.y, cr[e].a.z, cr[e].a.w, cr[e].b.x, cr[e].b.y, cr[e].b.z, cr[e].b.w,
                       cr[e].x.x};
        pass[e] = valid[e] && (!pf.use_sb || ScreenBoxOverlaps(bb, sb)) && BoxMayHit(bb, r);
        if (pass[e]) {
            int c0 = 0, c1 = pf.nc - 1, r0 = 0, r1 = pf.nr - 1;
            if (pf.use_sb) {
                // Columns whose fx interval can meet [sb.xlo, sb.xhi]; rows likewise.
                c0 = FirstAtLeast(sh.chi, pf.nc, sb.x, GuessIndex(sb.x, pf.fx_first, pf.fx_scale, pf.nc));
                c1 = LastAtMost(sh.clo, pf.nc, sb.y, GuessIndex(sb.y, pf.fx_first, pf.fx_scale, pf.nc) + 1);
                r0 = FirstAtLeast(sh.rhi, pf.nr, sb.z, GuessIndex(sb.z, pf.fy_first, pf.fy_scale, pf.nr));
                r1 = LastAtMost(sh.rlo, pf.nr, sb.w, GuessIndex(sb.w, pf.fy_first, pf.fy_scale, pf.nr) + 1);
            }
            pass[e] = c0 <= c1 && r0 <= r1;
            if (pass[e]) {
                npk[e] = static_cast<unsigned>((c1 - c0 + 1) * (r1 - r0 + 1));  // pixels of the range
                npk[e] = (npk[e] + kLanePixels - 1u) / kLanePixels;  // stream units: one lane's pixels
                bits[e] = (static_cast<unsigned>(r0) << 9) + (static_cast<unsigned>(c0) << 3) |
                          static_cast<unsigned>(c1 - c0 + 1) << 16 | static_cast<unsigned>(r1 - r0 + 1) << 24;
            }
        }
    }
    // Compact the survivors block-wide ((slice, wave, lane) order); exclusive packet prefix
    // in compacted order.
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
            sh.wave_n[e * W + wave] = __popcll(m);
            sh.wave_pk[e * W + wave] = incl[e];
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
        const unsigned wn = sh.wave_n[vw], wp = sh.wave_pk[vw];
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
            sh.sv0[slot] = cr[e].a;
            sh.sv1[slot] = cr[e].b;
            const float rnc = __builtin_amdgcn_rcpf(static_cast<float>((bits[e] >> 16) & 0xFFu));
            sh.sv2[slot] = make_float4(cr[e].x.x, cr[e].x.y, cr[e].x.z, rnc);
            sh.aux[slot] = make_uint2(pbase[e] + incl[e] - npk[e], bits[e]);
            const unsigned o = pbase[e] + incl[e] - 1u;  // the range's last pixel in the stream
            if (o < kWindowPixels) {                      // first window: its end bit
                atomicOr((o & 32u) ? &pkb[o >> 6].y : &pkb[o >> 6].x, 1u << (o & 31u));
            }
        }
    }
    if (tid == 0) {
        sh.aux[n_surv] = make_uint2(n_pk, 0u);
    }
    __syncthreads();
    // The other buffer (last read by the previous batch's walk, which every wave finished before
    // this batch's first barrier) is cleared for the next batch.
    if (tid < kWindowPackets) {
        sh.pk[buf ^ 1u][tid] = make_uint2(0u, 0u);
    }
    prefetch();
    // Walk the batch's pixel stream -- the survivors' ranges back to back in slot order, each
    // row-major -- in windows of kWindowPixels. Per window: a bitmap of the pixels that end a
    // survivor's range and, per 64-pixel packet, the number of ranges that end before it, so
    // that lane l of packet k (pixel g = 64 k + l) finds its survivor as that number plus the
    // range ends below it in the packet (mbcnt), and its pixel as position g - pre[s] of the
    // range. The waves split each window's packets evenly, kPacketIlp at a time (independent
    // chains; a tail repeats the last packet, harmless under the atomic min).
    constexpr int kPacketIlp = SRT_PACKET_ILP;
    const char* fxy = reinterpret_cast<const char*>(&sh.fxy[0][0]);
    char* keys = reinterpret_cast<char*>(&sh.keys[0][0]);
    const unsigned last_slot = n_surv == 0u ? 0u : n_surv - 1u;
    unsigned ended = 0u;  // ranges that end before the window (block-uniform)
#pragma unroll 1
    for (unsigned w0 = 0; w0 < n_pk; w0 += kWindowPixels) {
        const unsigned wn = min(kWindowPixels, n_pk - w0);
        const unsigned npk_w = (wn + kWave - 1u) / kWave;
        if (w0 != 0u) {  // a later window (rare: > kWindowPixels pixels in the batch): rebuild its bitmap
            __syncthreads();  // every wave done with the previous window
            if (tid < kWindowPackets) {
                pkb[tid] = make_uint2(0u, 0u);
            }
            __syncthreads();
            for (unsigned slot = tid; slot < n_surv; slot += kCullThreads) {
                const unsigned o = sh.aux[slot + 1].x - 1u - w0;  // the range's last pixel, in the window
                if (o < wn) {
                    atomicOr((o & 32u) ? &pkb[o >> 6].y : &pkb[o >> 6].x, 1u << (o & 31u));
                }
            }
            __syncthreads();
        }
        // Every wave: exclusive prefix of the range ends over the window's packets (2 per lane,
        // packets 2l and 2l + 1 in lane l), kept in registers -- no barrier to publish it.
        const uint2 pa = pkb[2 * lane], pb = pkb[2 * lane + 1];
        const unsigned ca = __popc(pa.x) + __popc(pa.y), cb = __popc(pb.x) + __popc(pb.y);
        unsigned incl = ca + cb;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const unsigned t = __shfl_up(incl, o);
            if (lane >= o) {
                incl += t;
            }
        }
        const unsigned za = ended + incl - ca - cb;  // ranges ending before packet 2 lane
        ended += static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(incl), kWave - 1));
        const unsigned k_begin = wave * npk_w / W, k_end = (wave + 1) * npk_w / W;
#pragma unroll 1
        for (unsigned k = k_begin; k < k_end; k += kPacketIlp) {
            PacketPixel px[kPacketIlp][kLanePixels];
            float4 ra[kPacketIlp], rb[kPacketIlp], rx[kPacketIlp];
            float2 f[kPacketIlp][kLanePixels];
#pragma unroll
            for (int u = 0; u < kPacketIlp; ++u) {
                const unsigned kk = min(k + u, k_end - 1u);
                // ranges ending before packet kk: lane kk / 2's prefix, plus its first packet's ends
                const int src = static_cast<int>(kk >> 1);
                unsigned z = static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(za), src));
                if (kk & 1u) {
                    z += static_cast<unsigned>(__builtin_amdgcn_readlane(static_cast<int>(ca), src));
                }
                const uint2 e = pkb[kk];  // one address: a broadcast read (from the scan's registers by
                                          // readlane: 2 VGPR spills in round 2, measured 3 % slower)
                const unsigned g = w0 + kk * kWave + static_cast<unsigned>(lane);
                const unsigned sl = min(__builtin_amdgcn_mbcnt_hi(e.y, __builtin_amdgcn_mbcnt_lo(e.x, 0u)) + z,
                                        last_slot);
                const bool in = g < n_pk;
                ra[u] = sh.sv0[sl];
                rb[u] = sh.sv1[sl];
                rx[u] = sh.sv2[sl];
                const uint2 ax = sh.aux[sl];
                const unsigned nc = (ax.y >> 16) & 0xFFu, nr = ax.y >> 24, base = ax.y & 0xFFFFu;
                const unsigned q = (g - ax.x) * kLanePixels;  // the lane's first pixel of the range, row-major
                // row = q / nc, exact: q < 1024 and 1 / nc within 1 ulp, so (q + 1/2) / nc is
                // >= 1/128 from an integer and the product is within 2^-10 of it
                const unsigned row = static_cast<unsigned>((static_cast<float>(q) + 0.5f) * rx[u].w);
                const unsigned col = q - __umul24(row, nc);
                // pixel q + j: j columns on, wrapping into the next rows (j < kLanePixels, so it
                // wraps at most j times); past the range's last row when the range's pixel count is
                // not a multiple of kLanePixels
#pragma unroll
                for (int j = 0; j < kLanePixels; ++j) {
                    unsigned c = col + j, r = row;
#pragma unroll
                    for (int w = 0; w < j; ++w) {
                        const bool wrap = c >= nc;
                        c = wrap ? c - nc : c;
                        r = wrap ? r + 1u : r;
                    }
                    const bool ok = in && r < nr;
                    px[u][j] = PacketPixel{ok ? base + (r << 9) + (c << 3) : 0u, ok};
                }
            }
            PacketHit h[kPacketIlp][kLanePixels];
#pragma unroll
            for (int u = 0; u < kPacketIlp; ++u) {
#pragma unroll
                for (int j = 0; j < kLanePixels; ++j) {
                    f[u][j] = *reinterpret_cast<const float2*>(fxy + px[u][j].pixb);
                }
            }
#pragma unroll
            for (int u = 0; u < kPacketIlp; ++u) {
#pragma unroll
                for (int j = 0; j < kLanePixels; ++j) {
                    h[u][j] = EvalPacket(ra[u], rb[u], rx[u], f[u][j], px[u][j].in);
                }
            }
#pragma unroll
            for (int u = 0; u < kPacketIlp; ++u) {
#pragma unroll
                for (int j = 0; j < kLanePixels; ++j) {
                    asm volatile("" ::"v"(h[u][j].key));
                }
            }
#pragma unroll
            for (int u = 0; u < kPacketIlp; ++u) {
#pragma unroll
                for (int j = 0; j < kLanePixels; ++j) {
                    if (h[u][j].hit) {
                        __hip_atomic_fetch_min(reinterpret_cast<unsigned long long*>(keys + px[u][j].pixb), h[u][j].key,
                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
                    }
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------
// Cull bins: the first cull level, built per band before the trace, in three launches (the
// frame's record setup rides in the second). A tile is 64 x 32 rays.
//   TileInfoKernel:     one block per tile reads the tile's sample offsets once: the ray box,
//                       "regular" (every offset equal to the first, bit for bit) and the first
//                       offset; it clears the tile's bin count and tags the frame if an offset
//                       lies outside [0, 1].
//   PrepareBinKernel:   per tile column and row, monotone bounds of the tile boxes (analytic for
//                       offsets in [0, 1], else reduced from the tile boxes: BinTileBounds); one
//                       thread per record (spatial order) computes the record and bins it.
//   WorkOrderKernel:    one block lists the trace work (BuildWorkOrder).
// Both steps drop only (record, tile) pairs that provably fail the exact test for every ray
// of the tile, so the frame stays bit-identical to brute force. A tile whose box is outside
// the screen-box range, or whose list overflowed, streams every record instead.
// ---------------------------------------------------------------------------------------
#ifndef SRT_BIN_THREADS
#define SRT_BIN_THREADS 256
#endif
constexpr int kBinThreads = SRT_BIN_THREADS;  // records per bin block = the band skip hint's unit (BlockExtentCount)
static_assert(kBinThreads % kWave == 0 && kPadTriangles % kBinThreads == 0, "bin block shape");
#ifndef SRT_LARGE_TILES
#define SRT_LARGE_TILES 16
#endif
constexpr int kLargeTiles = SRT_LARGE_TILES;  // records spanning more tiles go to the large list
static_assert(kLargeTiles <= 32, "a record's tile mask is 32 bits");
static_assert(kTileRows == kCullTileRows && kWave == kCullTileCols, "render.h tile shape");

struct BinParams {
    const float2* __restrict__ offsets;
    const CullRecord* __restrict__ cull;  // cull records in spatial order
    TileInfo* __restrict__ tile_info;
    unsigned* __restrict__ counts;      // tiles + 1 (the last one: large list)
    unsigned* __restrict__ lists;       // tiles x capacity
    unsigned* __restrict__ large_list;  // n_pad
    uint4* __restrict__ work;           // trace work list (BuildWorkOrder): 2 x uint4 per tile part
    unsigned* __restrict__ work_count;  // [0]: tile parts listed
    unsigned* __restrict__ range_tag;   // = gen: some sample offset of this frame lies outside [0, 1]
    unsigned gen;                       // frame number of the scene (never 0)
    unsigned capacity;
    unsigned descs;      // trace work descriptors the trace grid has room for (CullDescriptors)
    unsigned min_chunk;  // smallest candidate chunk of a split part
    unsigned n;
    unsigned exp;  // diagnostic build: experiment bits (env SRT_EXP), 0 in the product
    unsigned fused;  // tile info computed in the bin launch (CullFusedInfo): bins assume offsets in [0, 1]
    unsigned recompute;  // CullBins::recompute: screen boxes by position instead of cull records
    int tiles_x;
    int tiles_y;
    int width;
    int row_count;
    int row_begin;
    int row_interleave;
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

// One block per kInfoTiles vertically adjacent tiles: tiles (bx, kInfoTiles by + k), k = wave /
// kInfoWaves (a 64 x 16 tile alone is too little work for a 256-thread block: 4 loads per thread).
#ifndef SRT_INFO_TILES
#define SRT_INFO_TILES 2  // 4: one wave per tile, 510 blocks: tile info 5.2 -> 5.6 us, throughput +1 % (noise)
#endif
constexpr int kInfoTiles = SRT_INFO_TILES;
__device__ __forceinline__ void TileInfoBlock(const BinParams& p, int bx, int by) {
    constexpr int kWaves = kBinThreads / kWave;
    constexpr int kInfoWaves = kWaves / kInfoTiles;             // waves per tile
    constexpr int kPer = kTileRows / kInfoWaves;                 // offsets per thread (8)
    static_assert(kWaves % kInfoTiles == 0 && kTileRows % kInfoWaves == 0, "tile info block shape");
    __shared__ Box boxes[kWaves];
    __shared__ unsigned irregular[kInfoTiles];
    __shared__ unsigned out_of_range;
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const int sub = wave / kInfoWaves, w2 = wave % kInfoWaves;
    const int ty = by * kInfoTiles + sub;  // this wave's tile row (may be past the band: no write)
    const int x0 = bx * kWave;
    const int y0 = min(ty * kTileRows, p.row_count - 1);
    if (tid < kInfoTiles) {
        irregular[tid] = 0u;
    }
    if (tid == 0) {
        out_of_range = 0u;
    }
    // All loads first (clamped addresses: duplicates of real pixels), then the box. Same
    // expressions as GenerateRays, fx = fl(fl(x + ox) / W), but the division comes after the
    // reduction: the correctly rounded division by W > 0 is monotone, so the extremes of fx are the
    // quotients of the extremes of fl(x + ox), bit for bit (fl(x + ox) is never -0: x >= +0) -- two
    // divisions per tile instead of two per pixel. NaN positions drop out (fminf / fmaxf).
    const float2 o0 = p.offsets[static_cast<size_t>(y0) * p.width + x0];
    Box box{__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()};  // of the sums
    bool regular = true, in_range = true;
    auto take = [&](int x, int yy, float2 o) {
        const float sx = static_cast<float>(x) + o.x;
        const float sy = static_cast<float>(FrameRow(p.row_begin, p.row_interleave, yy)) + o.y;
        box = Box{fminf(box.xlo, sx), fmaxf(box.xhi, sx), fminf(box.ylo, sy), fmaxf(box.yhi, sy)};
        regular = regular && __float_as_uint(o.x) == __float_as_uint(o0.x) && __float_as_uint(o.y) == __float_as_uint(o0.y);
        in_range = in_range && o.x >= 0.f && o.x <= 1.f && o.y >= 0.f && o.y <= 1.f;  // NaN: false
    };
    if (x0 + kWave <= p.width && (p.width & 1) == 0 && (reinterpret_cast<uintptr_t>(p.offsets) & 15u) == 0) {
        // Whole-width tile, 16-B aligned rows: lane = a column pair of one of two rows, 16 B per
        // load (1 KB per wave instruction). (Nontemporal loads here measured 2.6 % slower.)
        const int xa = x0 + 2 * (lane & (kWave / 2 - 1)), half = lane / (kWave / 2);
        float4 o[kPer / 2];
#pragma unroll
        for (int k = 0; k < kPer / 2; ++k) {
            const int yy = min(y0 + (k * kInfoWaves + w2) * 2 + half, p.row_count - 1);
            o[k] = *reinterpret_cast<const float4*>(p.offsets + static_cast<size_t>(yy) * p.width + xa);
        }
#pragma unroll
        for (int k = 0; k < kPer / 2; ++k) {
            const int yy = min(y0 + (k * kInfoWaves + w2) * 2 + half, p.row_count - 1);
            take(xa, yy, make_float2(o[k].x, o[k].y));
            take(xa + 1, yy, make_float2(o[k].z, o[k].w));
        }
    } else {  // a tile at the frame's right edge or an odd width: 8-B loads, clamped columns
        const int xx = min(x0 + lane, p.width - 1);
        float2 o[kPer];
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            const int yy = min(y0 + w2 + k * kInfoWaves, p.row_count - 1);
            o[k] = p.offsets[static_cast<size_t>(yy) * p.width + xx];
        }
#pragma unroll
        for (int k = 0; k < kPer; ++k) {
            take(xx, min(y0 + w2 + k * kInfoWaves, p.row_count - 1), o[k]);
        }
    }
    box = WaveReduceBox(box);
    const bool wave_regular = __all(regular);
    const bool wave_in_range = __all(in_range) || ty >= p.tiles_y;  // a tile past the band: no tag
    __syncthreads();  // `irregular`, `out_of_range` initialised
    if (lane == 0) {
        boxes[wave] = box;
        if (!wave_regular) {
            irregular[sub] = 1u;
        }
        if (!wave_in_range) {
            out_of_range = 1u;
        }
    }
    __syncthreads();
    if (lane == 0 && w2 == 0 && ty < p.tiles_y) {  // the tile's first wave
        box = boxes[wave];
#pragma unroll
        for (int w = 1; w < kInfoWaves; ++w) {
            const Box b = boxes[wave + w];
            box = Box{fminf(box.xlo, b.xlo), fmaxf(box.xhi, b.xhi), fminf(box.ylo, b.ylo), fmaxf(box.yhi, b.yhi)};
        }
        box = Box{box.xlo / p.wf, box.xhi / p.wf, box.ylo / p.hf, box.yhi / p.hf};  // the rays' (fx, fy) box
        TileInfo ti;
        ti.box = make_float4(box.xlo, box.xhi, box.ylo, box.yhi);
        ti.ox = o0.x;
        ti.oy = o0.y;
        ti.regular = irregular[sub] == 0u ? 1u : 0u;
        ti.usable = ScreenBoxUsable(box) ? 1u : 0u;
        const unsigned tile = ty * p.tiles_x + bx;
        p.tile_info[tile] = ti;  // (the bin counts are reset by the work order that reads them)
    }
    if (tid == 0 && out_of_range != 0u) {
        *p.range_tag = p.gen;  // this frame's bin blocks reduce the tile boxes (BinTileBounds)
    }
}

using BinBatch = FrameArgs<BinParams>;
using BinTable = FrameTable<BinParams>;

template <class Frames>
__global__ __launch_bounds__(kBinThreads) void TileInfoKernel(const Frames batch) {
    TileInfoBlock(batch[blockIdx.z], blockIdx.x, blockIdx.y);
}

// Searches in a bin block's monotone tile bounds b[0..n) (lo' = .x, hi' = .y, both
// nondecreasing): an index guess from the linear model of the table (GuessIndex), then exact unit
// steps -- the bounds are near-linear in the tile index (analytic: fl(64 c / W)), so a search
// costs a step or two instead of a log2(n)-step bisection.
struct BoundModel {
    float first, scale;  // index ~ (v - first) * scale
};
__device__ __forceinline__ BoundModel MakeBoundModel(const float2* b, int n) {
    const float lo = b[0].x, hi = b[n - 1].y;
    return BoundModel{lo, n > 1 && hi > lo ? static_cast<float>(n) / (hi - lo) : 0.f};
}
// First index i with hi'[i] >= v (n if none).
__device__ __forceinline__ int FirstHiAtLeast(const float2* b, int n, float v, const BoundModel& m) {
    int g = min(max(GuessIndex(v, m.first, m.scale, n), 0), n);
    while (g > 0 && b[g - 1].y >= v) {
        --g;
    }
    while (g < n && b[g].y < v) {
        ++g;
    }
    return g;
}
// Last index i with lo'[i] <= v (-1 if none).
__device__ __forceinline__ int LastLoAtMost(const float2* b, int n, float v, const BoundModel& m) {
    int g = min(max(GuessIndex(v, m.first, m.scale, n) + 1, 0), n);  // guess of the first lo' > v
    while (g > 0 && b[g - 1].x > v) {
        --g;
    }
    while (g < n && b[g].x <= v) {
        ++g;
    }
    return g - 1;
}

// Trace work plan (WorkOrderKernel, after the bin kernel of a slot's first frame of a band shape;
// render.h CullBins::plan). One 32-B descriptor per trace block: a tile part, or one candidate
// chunk of a split part. The plan is scheduling only: a plan-only trace block (a frame that reuses
// the slot's plan) takes its part, chunk index, chunk count and split slot from it and everything
// it computes from its own frame's bins and tile info, so a plan made from any frame of the slot's
// band shape gives the same frame (the candidate counts of frames with offsets in [0, 1] do not
// depend on the offsets: analytic tile bounds), and that frame's pipeline is the bin launch and
// the trace. The grid has room for p.descs
// descriptors D; with P parts holding C candidates in all (each part counted with its tile's
// candidates), chunks of S = the power of two >= max(p.min_chunk, C / (D - P)) candidates fit,
// since sum ceil(c / S) <= P + C / S <= D. So the heavy parts -- which bound a frame's trace
// time -- are cut into several blocks and the light ones stay whole. The list is longest first
// (counting sort by the log2 of the candidates per descriptor, FULL-stream tiles first), so the
// heavy work starts first and the light work fills in behind it; order within a bucket is
// arbitrary (the frame does not depend on it). Descriptor: w0 = (tile part, its candidates, tile
// list length, flags), w1 = (sample offset x, y of the tile's first ray, chunk | chunks << 16,
// first split slot of the part); flags: 1 = every ray of the tile has that offset, 2 = FULL. A
// split part's chunks own consecutive split slots (key slices; the arrival counter at the first).
// A trace launched after this kernel (the same frame) takes the rest from the descriptor too, with
// flags 4 = empty (no candidate can hit a ray of the tile) and FULL also when the frame's bins are
// invalid; a plan-only trace (a later frame) reads those facts from its own bins (TraceParams::
// plan_only). The chunking is made as if every offset were in [0, 1], so it may serve later frames.
// (Gathering whole empty tiles four to a descriptor, one block storing all their misses, cut the
// trace grid by ~950 blocks at C3 and measured no faster: an empty part's block is cheap.)
// (BinParams::work_count: kOrderWords words, unused by the product kernels.)
constexpr int kOrderBuckets = 64;
constexpr int kOrderWords = 72;
constexpr unsigned kItemRegular = 1u;
constexpr unsigned kItemFull = 2u;
constexpr unsigned kItemEmpty = 4u;  // no candidate can hit a ray of the tile: every pixel misses
constexpr unsigned kWorkEnd = 0xFFFFFFFFu;  // w0.x of a descriptor past the end of the list
constexpr int kEmptyTest = 4;  // a tile with an empty bin list is tested against up to this many large-list records
struct OrderItem {
    unsigned cand, flags, parts;
};
__device__ __forceinline__ OrderItem MakeOrderItem(const BinParams& p, unsigned t, unsigned cnt, unsigned large,
                                                   const TileInfo& ti, bool bins_invalid) {
    OrderItem it;
    const bool full = ti.usable == 0u || cnt > p.capacity || bins_invalid;
    it.flags = (full ? kItemFull : 0u) | (ti.regular != 0u ? kItemRegular : 0u);
    it.cand = full ? 0u : cnt + large;
    const int rows_left = p.row_count - static_cast<int>(t / static_cast<unsigned>(p.tiles_x)) * kTileRows;
    it.parts = static_cast<unsigned>(min(kParts, (rows_left + kBlockRows - 1) / kBlockRows));
    return it;
}
// Chunks per part (chunk size 2^shift, at most kMaxChunks) and LPT bucket of a tile.
__device__ __forceinline__ void ItemChunks(unsigned cand, unsigned flags, unsigned shift, unsigned& nch,
                                           unsigned& bucket) {
    const bool full = (flags & kItemFull) != 0u;
    nch = full ? 1u : min(static_cast<unsigned>(kMaxChunks), max(1u, (cand + (1u << shift) - 1u) >> shift));
    const unsigned per = cand >> (31u - __builtin_clz(nch));  // ~ candidates per chunk
    bucket = full ? 63u : (per == 0u ? 0u : 32u - __builtin_clz(per));
}

// A bin block's monotone tile-column and tile-row bounds (lo' nondecreasing, hi' nondecreasing)
// into out[0 .. nx + ny) in LDS; `scratch` = 2 (nx + ny) LDS words; ends with a barrier.
//  * Every sample offset of the frame in [0, 1] (no tile block tagged the frame): tile column c
//    holds x in [64c, 64c + 63], so fl(x + o) lies in [64c, 64c + 64] and, the rounded division
//    being monotone, every fx of the tile in [fl(64c / W), fl((64c + 64) / W)]; rows likewise.
//    These analytic bounds contain every tile box and are already monotone: no reduction.
//  * Otherwise (offsets outside [0, 1], NaN): the usable tiles' boxes reduced per column and row
//    with LDS atomics on order-preserving bits, then made monotone (lo' = suffix minimum,
//    hi' = prefix maximum) by wave scans.
// Either way a tile outside a record's searched range cannot overlap its screen box; the tiles
// inside are tested against their own boxes, so the bins do not depend on which path ran.
__device__ void BinTileBounds(const BinParams& p, unsigned* scratch, float2* out) {
    const int tid = threadIdx.x;
    const int nthreads = blockDim.x;
    const int lane = tid & (kWave - 1);
    const int wave = tid / kWave;
    const int nx = p.tiles_x, ny = p.tiles_y;
    if (p.fused != 0u || *p.range_tag != p.gen) {  // tag: written by the previous launch's tile blocks
        for (int i = tid; i < nx + ny; i += nthreads) {
            const bool col = i < nx;
            const int r0 = FrameRow(p.row_begin, p.row_interleave, (i - nx) * kTileRows);  // the tile row's first
            const float v0 = col ? static_cast<float>(i * kWave) : static_cast<float>(r0);
            const float v1 = col ? static_cast<float>((i + 1) * kWave) : static_cast<float>(r0 + kTileRows);
            const float d = col ? p.wf : p.hf;
            out[i] = make_float2(v0 / d, v1 / d);
        }
        __syncthreads();
        return;
    }
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

// LDS of a bin block (dynamic, sized to the band so the bin blocks of one frame leave room for
// other frames' trace blocks): the tile bounds, then the histogram.
std::size_t BinLdsBytes(int nx, int ny) {
    const int hist = nx * ny > 2 * (nx + ny) ? nx * ny : 2 * (nx + ny);  // also BinTileBounds' scratch
    return static_cast<std::size_t>(nx + ny) * sizeof(float2) + static_cast<std::size_t>(hist) * sizeof(unsigned);
}

// Records and bins of a frame in one launch (the binned cull path). Block b owns spatial
// positions [256 b, 256 b + 256) (the scene's Morton order, so a block's records fall in few
// tiles; two records per thread, 98 VGPRs, measured 5 us slower). Each thread computes the record of its position (triangle order[i]) in registers and
// writes, by position, its quantized box (the FULL stream's input) and its 64-B cull record (the
// trace's only record reads), and its shading normal by id. The cull record is skipped when no
// trace of this band can read it: with every offset of the frame in [0, 1] (no tile block tagged
// it), every ray of a tile row of the band lies in that row's analytic bounds; a record whose
// quantized screen box meets none of the band's quantized tile-row bounds is never listed (its
// row range is empty) and never passes a FULL block's box test (a block box lies inside its tile
// row and quantisation is monotone). Padding and tagged frames write every record. The block then bins
// the records it holds: binary searches in the bounds give each record the range of tiles its
// screen box can overlap, every tile of the range passing ScreenBoxOverlaps + BoxMayHit against
// its own box gets the position appended (records spanning more than kLargeTiles tiles go to the
// large list). (Staging the block's window of tile boxes in LDS first, instead of each thread
// loading its tiles' boxes one after another, measured 1.4 us slower: two more barriers and a
// reduction for loads that hit the L2.) An LDS histogram of (tile, record) pairs reserves each touched tile's share of
// its list with ONE global atomic (per-pair global atomics serialise on the busy tiles).
// k / w and k % w for the bit index k < 32 of a record's tile range (w <= kLargeTiles): (k + 1/2) / w
// lies >= 1/(2w) from an integer, so the truncated float product is exact (the integer division
// was ~30 instructions per (record, tile) pair in each of the bin kernel's three tile loops).
struct RangeDiv {
    float inv_w;
    int w;
    __device__ __forceinline__ explicit RangeDiv(int width) : inv_w(width > 0 ? 1.0f / static_cast<float>(width) : 0.f), w(width) {}
    __device__ __forceinline__ int Row(int k) const { return static_cast<int>((static_cast<float>(k) + 0.5f) * inv_w); }
    __device__ __forceinline__ int Tile(int k, int r0, int c0, int nx) const {
        const int kr = Row(k);
        return (r0 + kr) * nx + c0 + (k - kr * w);
    }
};

// Whether any ray of the band can lie in the fy range [ylo, yhi] of a block of records (its screen
// boxes' union, LaunchBlockExtents), for a frame whose sample offsets all lie in [0, 1] (no range
// tag): a ray of frame row y has fy = fl(fl(y + sy) / H) in [fl(y / H), fl((y + 1) / H)] (the
// correctly rounded division is monotone), so rows below floor(ylo H) - 1 or above floor(yhi H) + 1
// end short of the range (1 / H is far above an ulp of fy). A block none of whose records' screen
// boxes meets a ray of the band has no record any ray of the band can hit (DESIGN.md section 5,
// exactness (ii)), so skipping it changes no pixel. Rows: a contiguous band's own; an interleaved or
// patterned band's whole 16-row tile rows (BandFrameRow), a superset.
__device__ __forceinline__ bool BandMayReach(const BinParams& p, float ylo, float yhi) {
    if (ylo > yhi) {
        return false;  // every record of the block is disabled (empty boxes)
    }
    if (!(ylo <= yhi)) {
        return true;  // NaN: no skip
    }
    const int h = static_cast<int>(p.hf);
    const double a = floor(static_cast<double>(ylo) * static_cast<double>(p.hf)) - 1.0;
    const double b = floor(static_cast<double>(yhi) * static_cast<double>(p.hf)) + 1.0;
    if (b < 0.0 || a > static_cast<double>(h - 1)) {
        return false;  // outside the frame's rows
    }
    const int ya = static_cast<int>(fmax(a, 0.0)), yb = static_cast<int>(fmin(b, static_cast<double>(h - 1)));
    const int every = p.row_interleave & 0xFFFF, g = p.row_interleave >> 16;
    if (every <= 1) {
        return yb >= p.row_begin && ya <= p.row_begin + p.row_count - 1;
    }
    const int t0 = p.row_begin / kCullTileRows, group = 1 << g;
    const int last = (p.row_count + kCullTileRows - 1) / kCullTileRows - 1;  // the band's last local tile row
    const int t_last = t0 + (last >> g) * every + (last & (group - 1));
    const int ta = max(ya / kCullTileRows, t0), tb = min(yb / kCullTileRows, t_last);
    for (int t = ta; t <= tb && t < ta + every; ++t) {
        if ((t - t0) % every < group) {
            return true;
        }
    }
    return false;
}

// The block extents (render.h LaunchBlockExtents): block b's records computed as PrepareBinKernel
// computes them (vertices by position, the one-piece screen box, whose y half ComputeRecordY
// reproduces bit for bit: screen_box.h), reduced to (min ylo, max yhi); a NaN box end widens the
// block to everything.
__global__ __launch_bounds__(kBinThreads) void BlockExtentKernel(PrepareParams pp, float2* __restrict__ ext) {
    __shared__ float part[2][kBinThreads / kWave];
    const unsigned i = blockIdx.x * kBinThreads + threadIdx.x;
    float lo = __builtin_inff(), hi = -__builtin_inff();
    if (i < pp.n_pad) {
        const bool real = i < pp.n;
        float c[9], vol;
        float4 sb;
        ComputeRecord(pp, pp.svertices + static_cast<size_t>(kSpatialStride) * (real ? i : 0u), real, c, vol, sb);
        lo = sb.z == sb.z ? sb.z : -__builtin_inff();
        hi = sb.w == sb.w ? sb.w : __builtin_inff();
    }
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        lo = fminf(lo, __shfl_xor(lo, o));
        hi = fmaxf(hi, __shfl_xor(hi, o));
    }
    const int wave = threadIdx.x / kWave;
    if ((threadIdx.x & (kWave - 1)) == 0) {
        part[0][wave] = lo;
        part[1][wave] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int w = 1; w < kBinThreads / kWave; ++w) {
            lo = fminf(lo, part[0][w]);
            hi = fmaxf(hi, part[1][w]);
        }
        ext[blockIdx.x] = make_float2(lo, hi);
    }
}

struct PrepareBinParams {
    PrepareParams prep;
    BinParams bin;
};
using PrepareBinBatch = FrameArgs<PrepareBinParams>;
using PrepareBinTable = FrameTable<PrepareBinParams>;
#ifndef SRT_BIN_AHEAD
#define SRT_BIN_AHEAD 4
#endif
constexpr int kBinAhead = SRT_BIN_AHEAD;  // tile boxes a bin thread loads at once
// BAND: a band short of the whole frame (the tile info ran first, `fused` is 0): the x half of a
// record's screen box waits for its band test (ComputeRecordY). Full frames take ComputeRecord.
template <class Frames, bool BAND>
__global__ __launch_bounds__(kBinThreads) void PrepareBinKernel(const Frames batch) {
    extern __shared__ float2 bin_lds[];
    const PrepareBinParams& pb = batch[blockIdx.z];
    const BinParams& p = pb.bin;
    const PrepareParams& pp = pb.prep;
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 0);
    if (p.fused != 0u) {  // the blocks past the record blocks compute the tile info (CullFusedInfo)
        const unsigned rec_blocks = (pp.n_pad + kBinThreads - 1) / kBinThreads;
        if (blockIdx.x >= rec_blocks) {
            const unsigned k = blockIdx.x - rec_blocks;
            TileInfoBlock(p, static_cast<int>(k % static_cast<unsigned>(p.tiles_x)),
                          static_cast<int>(k / static_cast<unsigned>(p.tiles_x)));
            SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 1);
            return;
        }
    }
    const int tid = threadIdx.x;
    if constexpr (BAND) {
        // A block of records that cannot reach the band's rows (LaunchBlockExtents' skip hint; frames
        // whose offsets all lie in [0, 1]) leaves only its quantized boxes, empty, for the FULL stream.
        if (pp.block_ext != nullptr && *p.range_tag != p.gen) {
            const float2 e = pp.block_ext[blockIdx.x];
            if (!BandMayReach(p, e.x, e.y)) {
                const unsigned i = blockIdx.x * kBinThreads + tid;
                if (i < pp.n_pad) {
                    pp.qboxes[i] = QuantizeBox(
                        make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff()));
                }
                return;
            }
        }
    }
    const int nx = p.tiles_x, ny = p.tiles_y;
    const int tiles = nx * ny;
    float2* b = bin_lds;
    unsigned* hist = reinterpret_cast<unsigned*>(bin_lds + nx + ny);
    __shared__ unsigned bin_span[2];  // the block's lowest and highest binned tile (ordered by BinTileBounds' barrier)
    if (tid == 0) {
        bin_span[0] = ~0u;
        bin_span[1] = 0u;
    }

    // This thread's record (its loads in flight while the block builds the tile bounds).
    const unsigned i = blockIdx.x * kBinThreads + tid;  // spatial-order position (list entry)
    const bool real = i < pp.n;
    float c[9], vol = 0.f;
    float4 sb = make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff());
    // by position (render.h kSpatialStride): the vertices and the id, no order -> vertex chain
    const float* v = pp.svertices + static_cast<size_t>(kSpatialStride) * (real ? i : 0u);
    const unsigned id = real ? __float_as_uint(v[9]) : i;
    BoxSolve bs;
    bool xpend = false;
    if (i < pp.n_pad) {
        if constexpr (BAND) {
            ComputeRecordY(pp, v, real, c, vol, sb, bs, xpend);
        } else {
            ComputeRecord(pp, v, real, c, vol, sb);
        }
    }
    // The monotone tile-column and tile-row bounds (the histogram's LDS is the reduction's
    // scratch), then the histogram zeroed.
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 1);
    BinTileBounds(p, hist, b);
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 2);
    if (i < pp.n_pad) {
        bool needed = !real || p.fused != 0u || *p.range_tag == p.gen;  // fused: a full frame, every record
        if (!needed) {  // does the quantized box meet a tile row of the band (analytic row bounds)?
            // Quantisation keeps both bound sequences nondecreasing: the first row whose quantized
            // hi reaches the box's lo has the smallest lo of the rows that can meet it.
            const int qlo = QuantLo(sb.z), qhi = QuantHi(sb.w);
            int lo = 0, hi = ny;
            while (lo < hi) {
                const int mid = (lo + hi) >> 1;
                if (QuantHi(b[nx + mid].y) >= qlo) {
                    hi = mid;
                } else {
                    lo = mid + 1;
                }
            }
            needed = lo < ny && QuantLo(b[nx + lo].x) <= qhi;
        }
        // The x half of the box for records the band can see; the others get the empty box (their
        // y extent meets no tile row of the band, so no box test of the band could pass either).
        if constexpr (BAND) {
            if (xpend && needed) {
                ScreenBoxX(bs, sb.x, sb.y);
            } else if (xpend) {
                sb = make_float4(__builtin_inff(), -__builtin_inff(), __builtin_inff(), -__builtin_inff());
            }
        }
        pp.qboxes[i] = QuantizeBox(sb);
        if (needed && p.recompute != 0u) {
            pp.screen_boxes[i] = sb;  // by position: the trace recomputes the rest (TraceRecords<true>)
        } else if (needed) {
            CullRecord r;
            r.a = make_float4(c[0], c[1], c[2], c[3]);
            r.b = make_float4(c[4], c[5], c[6], c[7]);
            r.x = make_float4(c[8], vol, __uint_as_float(id), 0.f);
            r.sb = sb;
            pp.cull[i] = r;
        }
    }

    // The record's tile range (bit k of the mask below = tile (r0 + k / w, c0 + k % w) of the
    // range, at most kLargeTiles of them).
    int c0 = 0, r0 = 0, w = 0, h = 0;
    if (real && sb.x <= sb.y && sb.z <= sb.w && !SRT_EXP_BIT(p, 1u)) {  // else disabled: empty box
        // Any tile (c, r) whose box overlaps sb has hi'[c] >= hi[c] >= sb.xlo and
        // lo'[c] <= lo[c] <= sb.xhi, so c lies in [c0, c1]; rows likewise.
        const BoundModel mc = MakeBoundModel(b, nx), mr = MakeBoundModel(b + nx, ny);
        int c1, r1;
        if (SRT_EXP_BIT(p, 16u)) {  // diag timing: a fixed one-tile range instead of the searches
            c0 = c1 = r0 = r1 = static_cast<int>(i % 4u);
        } else {
            c0 = FirstHiAtLeast(b, nx, sb.x, mc);
            c1 = LastLoAtMost(b, nx, sb.y, mc);
            r0 = FirstHiAtLeast(b + nx, ny, sb.z, mr);
            r1 = LastLoAtMost(b + nx, ny, sb.w, mr);
        }
        w = max(c1 - c0 + 1, 0);
        h = max(r1 - r0 + 1, 0);
        if (w * h > kLargeTiles && !SRT_EXP_BIT(p, 2u)) {
            p.large_list[atomicAdd(&p.counts[tiles], 1u)] = i;
            if (p.recompute != 0u) {
                // the whole record of a large-list entry: the empty tests read it (WorkOrderKernel,
                // plan-only traces)
                CullRecord r;
                r.a = make_float4(c[0], c[1], c[2], c[3]);
                r.b = make_float4(c[4], c[5], c[6], c[7]);
                r.x = make_float4(c[8], vol, __uint_as_float(id), 0.f);
                r.sb = sb;
                pp.cull[i] = r;
            }
        }
    }
    const bool listed = w * h > 0 && w * h <= kLargeTiles && !SRT_EXP_BIT(p, 2u);
    const RangeDiv rd(w);
    unsigned mask = 0u;
    if (listed) {
        const Record rec{c[0], c[1], c[2], c[3], c[4], c[5], c[6], c[7], c[8]};
        // The first kBinAhead tiles' boxes are loaded together (most ranges are a few tiles), the
        // rest one after another.
        float4 box[kBinAhead];
        unsigned usable[kBinAhead];
#pragma unroll
        for (int k = 0; k < kBinAhead; ++k) {
            const int kc = min(k, w * h - 1);
            const int kr = rd.Row(kc);
            if (p.fused != 0u) {  // the analytic tile box (contains the tile's rays for offsets in [0, 1])
                const float2 bx = b[c0 + kc - kr * w], by = b[nx + r0 + kr];
                box[k] = make_float4(bx.x, bx.y, by.x, by.y);
                usable[k] = 1u;
            } else {
                const TileInfo& ti = p.tile_info[(r0 + kr) * nx + c0 + kc - kr * w];
                box[k] = ti.box;
                usable[k] = ti.usable;
            }
        }
#pragma unroll
        for (int k = 0; k < kBinAhead; ++k) {
            const Box tb{box[k].x, box[k].y, box[k].z, box[k].w};
            if (k < w * h && usable[k] != 0u && (SRT_EXP_BIT(p, 32u) || (ScreenBoxOverlaps(tb, sb) && BoxMayHit(tb, rec)))) {
                mask |= 1u << k;
            }
        }
#pragma unroll 1
        for (int k = kBinAhead; k < w * h; ++k) {
            Box tb;
            unsigned use = 1u;
            const int kr = rd.Row(k);
            if (p.fused != 0u) {
                const float2 bx = b[c0 + k - kr * w], by = b[nx + r0 + kr];
                tb = Box{bx.x, bx.y, by.x, by.y};
            } else {
                const TileInfo ti = p.tile_info[(r0 + kr) * nx + c0 + k - kr * w];
                tb = Box{ti.box.x, ti.box.y, ti.box.z, ti.box.w};
                use = ti.usable;
            }
            if (use != 0u && ScreenBoxOverlaps(tb, sb) && BoxMayHit(tb, rec)) {
                mask |= 1u << k;
            }
        }
    }
    // The block's tile span: its records are spatial neighbours (Morton order), so the tiles they
    // are binned to lie in a few tile rows -- the histogram is zeroed and scanned only there (a
    // pass over every tile per block was O(blocks x tiles): 3907 x 8100 at C5).
    unsigned t_lo = mask != 0u ? static_cast<unsigned>(rd.Tile(__builtin_ctz(mask), r0, c0, nx)) : ~0u;
    unsigned t_hi = mask != 0u ? static_cast<unsigned>(rd.Tile(31 - __builtin_clz(mask), r0, c0, nx)) : 0u;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        t_lo = min(t_lo, static_cast<unsigned>(__shfl_xor(static_cast<int>(t_lo), o)));
        t_hi = max(t_hi, static_cast<unsigned>(__shfl_xor(static_cast<int>(t_hi), o)));
    }
    if ((tid & (kWave - 1)) == 0) {
        atomicMin(&bin_span[0], t_lo);
        atomicMax(&bin_span[1], t_hi);
    }
    __syncthreads();
    t_lo = bin_span[0];
    t_hi = bin_span[1];
    const unsigned span_n = t_lo <= t_hi ? t_hi - t_lo + 1u : 0u;  // no listed record: empty
    for (unsigned k = static_cast<unsigned>(tid); k < span_n; k += kBinThreads) {
        hist[t_lo + k] = 0u;
    }
    __syncthreads();  // the span's histogram zeroed
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 3);
    for (unsigned m = SRT_EXP_BIT(p, 8u) ? 0u : mask; m != 0u; m &= m - 1u) {  // diag timing: 8 skips the counts
        const int k = __builtin_ctz(m);
        atomicAdd(&hist[rd.Tile(k, r0, c0, nx)], 1u);
    }
    __syncthreads();
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 4);
    for (unsigned k = static_cast<unsigned>(tid); k < span_n; k += kBinThreads) {
        const unsigned t = t_lo + k;
        const unsigned h = hist[t];
        if (h != 0u) {
            hist[t] = SRT_EXP_BIT(p, 4u) ? 0u : atomicAdd(&p.counts[t], h);  // this block's base in the list
        }
    }
    __syncthreads();
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 5);
    for (unsigned m = mask; m != 0u; m &= m - 1u) {
        const int k = __builtin_ctz(m);
        const unsigned t = static_cast<unsigned>(rd.Tile(k, r0, c0, nx));
        const unsigned at = atomicAdd(&hist[t], 1u);
        if (at < p.capacity) {
            p.lists[static_cast<size_t>(t) * p.capacity + at] = i;
        }
    }
#ifdef SRT_DIAG
    __syncthreads();
    SRT_SETUP_MARK(kDiagBinRow + blockIdx.x, 6);
#endif
}

// The trace work list after the bin kernel: one 256-thread block per 256 tiles. Every block reads
// every tile's list length and flags (8 KB of counts, 16 KB of tile flags at 1080p: cheap next to
// the serial latency of one block doing it all, ~9 us), so every block knows the frame's chunk size,
// the whole longest-first counting sort's bucket bases and how many descriptors and split slots the
// tiles of the blocks before it take, without waiting for another block: each places its own tiles'
// descriptors and writes its share of the end marks with no global atomic, and the trace blocks
// reset the bin counts they consume. (Per-bucket global cursors plus a last-block reset, this
// kernel's first multi-block form: 11.0 us one frame in flight, three dependent atomic round trips.)
constexpr int kOrderBlock = 256;
constexpr int kOrderTilesPerThread = 8;  // tiles' loads in flight per thread (one pass at 1080p: 2040 tiles)
#ifndef SRT_ORDER_COPIES
#define SRT_ORDER_COPIES 16
#endif
constexpr int kOrderCopies = SRT_ORDER_COPIES;  // LDS copies of the bucket histograms (lane l: copy l % copies)
constexpr int kOrderStride = kOrderBuckets + 1;  // words per copy: the copies of one bucket in different banks
template <class Frames>
__global__ __launch_bounds__(kOrderBlock) void WorkOrderKernel(const Frames batch) {
    const BinParams& p = batch[blockIdx.z];
    __shared__ CullRecord lrec[kEmptyTest];
    __shared__ unsigned hist8[kOrderCopies][kOrderStride];    // descriptors per bucket (the frame)
    __shared__ unsigned before8[kOrderCopies][kOrderStride];  // ... of the tiles of earlier blocks
    __shared__ unsigned hist[kOrderBuckets];    // this block's first descriptor per bucket
    __shared__ unsigned local[kOrderBuckets];   // this block's descriptors per bucket
    __shared__ unsigned sums[4];  // candidates / 16, parts, this block's split slots, earlier blocks' slots
    extern __shared__ unsigned order_lds[];     // per tile: candidates, then flags | parts << 2 (bytes)
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const unsigned tiles = static_cast<unsigned>(p.tiles_x * p.tiles_y);
    const unsigned first = blockIdx.x * kOrderBlock;  // this block's tiles: [first, first + kOrderBlock)
    unsigned* cnt = order_lds;
    unsigned char* meta = reinterpret_cast<unsigned char*>(order_lds + tiles);
    SRT_SETUP_MARK(kDiagOrderRow + blockIdx.x, 0);
    // The loads on the block's critical path first -- every tile's list length and flags, this
    // thread's own tile's info (its descriptor), the large list's length --, the rest after them
    // (the large list's first records, read after the items: a dependent chain of three round
    // trips that would otherwise delay the tiles' loads).
    constexpr int kU = kOrderTilesPerThread;
    unsigned c[kU], cn[kU];
    uint2 ru[kU], rn[kU];  // (regular, usable)
    auto load_step = [&](unsigned t0, unsigned (&cc)[kU], uint2 (&rr)[kU]) {
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const unsigned t = min(t0 + u * kOrderBlock, tiles - 1u);
            cc[u] = p.counts[t];
            rr[u] = *reinterpret_cast<const uint2*>(&p.tile_info[t].regular);
        }
    };
    load_step(tid, c, ru);
    const unsigned mine = first + static_cast<unsigned>(tid);
    const TileInfo my_ti = p.tile_info[min(mine, tiles - 1u)];
    const unsigned large = p.counts[tiles];
    // A fused launch binned with the analytic tile bounds, which hold only for offsets in [0, 1]:
    // if a tile-info block found one outside (the range tag), every tile streams every record (its
    // descriptors say FULL). The plan itself is made as if the offsets were in range: it may serve
    // the slot's later frames.
    const bool bins_invalid = p.fused != 0u && *p.range_tag == p.gen;
    if (tid < kOrderBuckets) {
        local[tid] = 0u;
    }
    for (int k = tid; k < kOrderCopies * kOrderStride; k += kOrderBlock) {
        (&hist8[0][0])[k] = 0u;
        (&before8[0][0])[k] = 0u;
    }
    if (tid < 4) {
        sums[tid] = 0u;
    }
    // (1) every tile's item into LDS, the frame's candidate and part totals; the next step's loads
    // are issued before this step's items are made (4K frames: 8100 tiles, four steps of 2048, whose
    // load round trips would otherwise follow one another)
    unsigned long long my_cand = 0ull;
    unsigned my_parts = 0u;
    for (unsigned t0 = tid; t0 < tiles; t0 += kU * kOrderBlock) {
        const unsigned next = t0 + kU * kOrderBlock;
        if (next < tiles) {
            load_step(next, cn, rn);
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const unsigned t = t0 + u * kOrderBlock;
            if (t < tiles) {
                TileInfo ti{};
                ti.regular = ru[u].x;
                ti.usable = ru[u].y;
                const OrderItem it = MakeOrderItem(p, t, c[u], large, ti, false);
                cnt[t] = it.cand;
                meta[t] = static_cast<unsigned char>(it.flags | it.parts << 2);
                my_cand += static_cast<unsigned long long>(it.parts) * it.cand;
                my_parts += it.parts;
            }
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            c[u] = cn[u];
            ru[u] = rn[u];
        }
    }
    if (tid < kEmptyTest && static_cast<unsigned>(tid) < large && large <= static_cast<unsigned>(kEmptyTest)) {
        lrec[tid] = p.cull[p.large_list[tid]];  // read after the barriers below
    }
    unsigned v16 = static_cast<unsigned>((my_cand + 15ull) >> 4), vp = my_parts;
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        v16 += __shfl_xor(v16, o);
        vp += __shfl_xor(vp, o);
    }
    __syncthreads();  // hist / before / local / sums zeroed
    SRT_SETUP_MARK(kDiagOrderRow + blockIdx.x, 1);
    if (lane == 0) {
        atomicAdd(&sums[0], v16);
        atomicAdd(&sums[1], vp);
    }
    __syncthreads();
    SRT_SETUP_MARK(kDiagOrderRow + blockIdx.x, 2);
    // (2) chunk size S = the power of two >= max(min_chunk, C / (D - P)), so that sum ceil(c / S)
    // <= P + C / S <= D fits the grid; the frame's bucket histogram (longest first), and the
    // descriptors and split slots of the tiles before this block's: every block derives the same
    // counting sort from the same LDS copy, so its tiles' places need no global atomics.
    unsigned shift = 31u;
    if (p.descs > sums[1]) {
        const unsigned room = p.descs - sums[1];
        const unsigned long long want = (16ull * sums[0] + room - 1ull) / room;
        const unsigned long long size = want > p.min_chunk ? want : p.min_chunk;
        shift = size >= (1ull << 31) ? 31u : 64u - static_cast<unsigned>(__builtin_clzll(size - 1ull));
        shift = size <= 1ull ? 0u : shift;
    }
    // The frame's histogram and the earlier blocks' share in kOrderCopies LDS copies, lane l adding
    // to copy l % kOrderCopies, summed after the barrier: most tiles fall in a few buckets, and the
    // lanes adding to one word serialise (one copy: ~3.7 us of this kernel's ~9 us one frame in
    // flight); the copies are kOrderStride = 65 words apart, so one bucket's copies lie in
    // different banks. A thread's kU tiles' items are read from LDS together.
    unsigned my_n = 0u, my_nch = 1u, my_bucket = 0u, slots_before = 0u;
    const unsigned copy = static_cast<unsigned>(lane) % kOrderCopies;
    for (unsigned t0 = tid; t0 < tiles; t0 += kU * kOrderBlock) {
        unsigned m[kU], cc[kU];
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const unsigned t = t0 + u * kOrderBlock;
            m[u] = t < tiles ? meta[t] : 0u;
            cc[u] = t < tiles ? cnt[t] : 0u;
        }
#pragma unroll
        for (int u = 0; u < kU; ++u) {
            const unsigned t = t0 + u * kOrderBlock;
            const unsigned parts = m[u] >> 2;
            if (parts != 0u) {
                unsigned nch, bucket;
                ItemChunks(cc[u], m[u] & 3u, shift, nch, bucket);
                const unsigned n = parts * nch;
                atomicAdd(&hist8[copy][bucket], n);
                if (t < first) {
                    atomicAdd(&before8[copy][bucket], n);
                    slots_before += nch > 1u ? n : 0u;
                } else if (t == mine) {
                    my_n = n;
                    my_nch = nch;
                    my_bucket = bucket;
                }
            }
        }
    }
#pragma unroll
    for (int o = 1; o < kWave; o <<= 1) {
        slots_before += __shfl_xor(slots_before, o);
    }
    if (lane == 0 && slots_before != 0u) {
        atomicAdd(&sums[3], slots_before);
    }
    const unsigned my_at = my_n != 0u ? atomicAdd(&local[my_bucket], my_n) : 0u;  // place in this block's share
    const unsigned my_slot = my_nch > 1u ? atomicAdd(&sums[2], my_n) : 0u;
    __syncthreads();
    if (tid < kWave) {  // bucket b's first descriptor: those of the heavier buckets (suffix sum, exclusive)
        unsigned c = 0u, bf = 0u;
#pragma unroll
        for (int k = 0; k < kOrderCopies; ++k) {
            c += hist8[k][lane];
            bf += before8[k][lane];
        }
        unsigned suf = c;
#pragma unroll
        for (int o = 1; o < kWave; o <<= 1) {
            const unsigned u = __shfl_down(suf, o);
            suf += lane + o < kWave ? u : 0u;
        }
        hist[lane] = suf - c + bf;  // this block's first descriptor in bucket `lane`
        if (lane == 0) {
            sums[0] = suf;  // descriptors listed
        }
    }
    __syncthreads();
    SRT_SETUP_MARK(kDiagOrderRow + blockIdx.x, 3);
    const unsigned used = sums[0];
    // (3) this thread's tile's descriptors
    if (my_n != 0u) {
        const unsigned t = mine;
        const unsigned at = hist[my_bucket] + my_at;
        const unsigned slot = my_nch > 1u ? sums[3] + my_slot : 0u;
        const unsigned flags = meta[t] & 3u, cand = cnt[t], parts = meta[t] >> 2;
        const unsigned list_len = (flags & kItemFull) ? 0u : cand - large;
        // This frame's facts (read by a trace of this launch; a plan-only trace reads its own):
        // FULL when the bins are invalid, and empty when the bin list is empty and none of the
        // few large-list records can hit a ray of the tile box (the tests the trace blocks run
        // against their part boxes, which lie inside it: every pixel misses; a ray outside the box
        // has a NaN position and misses too).
        unsigned out_flags = flags | (bins_invalid ? kItemFull : 0u);
        if ((out_flags & kItemFull) == 0u && list_len == 0u && large <= static_cast<unsigned>(kEmptyTest)) {
            const Box tb{my_ti.box.x, my_ti.box.y, my_ti.box.z, my_ti.box.w};
            bool may = false;
            for (unsigned k = 0; k < large; ++k) {
                const CullRecord& r = lrec[k];
                const Record q{r.a.x, r.a.y, r.a.z, r.a.w, r.b.x, r.b.y, r.b.z, r.b.w, r.x.x};
                may = may || (ScreenBoxOverlaps(tb, r.sb) && BoxMayHit(tb, q));
            }
            out_flags |= may ? 0u : kItemEmpty;
        }
        for (unsigned part = 0; part < parts; ++part) {
            for (unsigned ch = 0; ch < my_nch; ++ch) {
                const unsigned d = at + part * my_nch + ch;
                p.work[2 * d] = make_uint4(t * kParts + part, cand, list_len, out_flags);
                p.work[2 * d + 1] = make_uint4(__float_as_uint(my_ti.ox), __float_as_uint(my_ti.oy), ch | my_nch << 16,
                                               slot + part * my_nch);
            }
        }
    }
    // descriptors past the list: end marks (every block a share; a trace block reads nothing first)
    for (unsigned d = used + first + static_cast<unsigned>(tid); d < p.descs; d += gridDim.x * kOrderBlock) {
        p.work[2 * d] = make_uint4(kWorkEnd, 0u, 0u, 0u);
    }
#ifdef SRT_DIAG
    __syncthreads();
    SRT_SETUP_MARK(kDiagOrderRow + blockIdx.x, 4);
#endif
    // (the bin counts are reset by the trace blocks that consume these descriptors)
}

std::size_t OrderLdsBytes(int tiles) { return static_cast<std::size_t>(tiles) * 5 + 16; }

#ifndef SRT_TRACE_OCC
#define SRT_TRACE_OCC 6
#endif

// Where a trace block's candidate records come from. RC = false: the 64-B cull record by position
// (written by the record pass: LaunchPrepare, or the bin kernel of a stored-record launch).
// RC = true (a binned launch with CullBins::recompute): the bin kernel writes only the screen box
// by position, and the trace recomputes the edge coefficients and vol from the vertices by position
// with the record pass's own ComputeEdges under the same frame vectors -- the same bits -- and
// takes the id from the spatial order (a padding position is its own id, >= n: a disabled record).
struct RawRecord {
    float v[9];
    unsigned id;
    float4 sb;
};
template <bool RC>
struct TraceRecords {
    using Raw = CullRecord;
    static __device__ __forceinline__ Raw Load(const TraceParams& p, unsigned pos) { return p.cull[pos]; }
    static __device__ __forceinline__ CullRecord Make(const TraceParams&, const Raw& r) { return r; }
};
template <>
struct TraceRecords<true> {
    using Raw = RawRecord;
    static __device__ __forceinline__ Raw Load(const TraceParams& p, unsigned pos) {
        Raw r;
        const bool real = pos < p.n;
        const float4* v = reinterpret_cast<const float4*>(p.svertices + static_cast<size_t>(kSpatialStride) * (real ? pos : 0u));
        const float4 v0 = v[0], v1 = v[1], v2 = v[2];
        r.v[0] = v0.x, r.v[1] = v0.y, r.v[2] = v0.z, r.v[3] = v0.w;
        r.v[4] = v1.x, r.v[5] = v1.y, r.v[6] = v1.z, r.v[7] = v1.w;
        r.v[8] = v2.x;
        r.id = real ? __float_as_uint(v2.y) : pos;
        r.sb = p.screen_boxes[pos];
        return r;
    }
    static __device__ __forceinline__ CullRecord Make(const TraceParams& p, const Raw& r) {
        float c[9], vol;
        ComputeEdges(p.eye, p.base, p.du, p.dv, r.v, r.id < p.n, c, vol);
        CullRecord cr;
        cr.a = make_float4(c[0], c[1], c[2], c[3]);
        cr.b = make_float4(c[4], c[5], c[6], c[7]);
        cr.x = make_float4(c[8], vol, __uint_as_float(r.id), 0.f);
        cr.sb = r.sb;
        return cr;
    }
};

template <class Frames, bool RC = false>
__global__ __launch_bounds__(kCullThreads, SRT_TRACE_OCC) void TraceCullKernel(const Frames batch) {
    const TraceParams& p = batch[blockIdx.z];
    using Recs = TraceRecords<RC>;
    constexpr int R = kCullR;
    __shared__ CullShared sh;
#ifdef SRT_DIAG
    const unsigned long long d_rt0 = __builtin_amdgcn_s_memrealtime();
    const unsigned d_blk = (blockIdx.z * gridDim.y + blockIdx.y) * gridDim.x + blockIdx.x;
    unsigned long long d_gather = 0, d_walk = 0, d_batches = 0, d_cand = 0;
    unsigned long long d_mark = __builtin_amdgcn_s_memtime();
    auto diag_end = [&](unsigned it, unsigned ch, unsigned nch, unsigned last, unsigned full, unsigned fl) {
        if (threadIdx.x == 0 && d_blk < kDiagBlocks) {
            unsigned long long* d = g_srt_diag[d_blk];
            d[1] = d_gather;
            d[2] = d_walk;
            d[5] = d_batches;
            d[7] = (full ? 0ull : 8ull) | d_cand << 40;
            d[8] = d_rt0;
            d[9] = __builtin_amdgcn_s_memrealtime();
            d[10] = it;
            d[11] = ch | nch << 16 | static_cast<unsigned long long>(last) << 32;
            d[12] = fl | static_cast<unsigned long long>(blockIdx.z) << 32;
        }
    };
#define SRT_DIAG_END(it, ch, nch, last, full) diag_end(it, ch, nch, last, full, flags)
#else
#define SRT_DIAG_END(it, ch, nch, last, full)
#endif
    // Block = one part (kBlockRows rows) of a cull tile. Binned: work item blockIdx.x of the
    // tile order's list (a part, or one candidate chunk of a split part; the grid is sized for
    // the longest list and the blocks past its end exit). Unbinned: part (x, y), FULL stream.
    unsigned item, chunk = 0u, nchunks = 1u, slot = 0u, flags = kItemFull;
    float ox = 0.f, oy = 0.f;
    CullSource src{nullptr, nullptr, 0u, 0u, 0u, true};
    if (p.work != nullptr) {
        // The work list (WorkOrderKernel) gives this block its tile part and chunk; with an order
        // launch for this frame it also holds the frame's facts, else it is the slot's plan
        // (scheduling only) and the block reads them from the frame's bins and tile info.
        const unsigned d = blockIdx.x;  // < descs: the plan, then end marks
        const uint4 w0 = p.work[2 * d], w1 = p.work[2 * d + 1];
        if (w0.x == kWorkEnd) {
            return;
        }
        item = w0.x;
        chunk = w1.z & 0xFFFFu;
        nchunks = max(w1.z >> 16, 1u);
        slot = w1.w;
        const unsigned t = item / kParts;
        // The slot's next frame bins into the other count buffer: each tile's count reset by its
        // first part's first chunk, the large list's by the first descriptor.
        if (threadIdx.x == 0 && chunk == 0u && item % kParts == 0u) {
            p.bin_counts_next[t] = 0u;
        }
        if (threadIdx.x == 0 && d == 0u) {
            p.bin_counts_next[p.tiles] = 0u;
        }
        bool full;
        unsigned c_t, list_len;
        if (p.plan_only != 0u) {
            // This frame's facts, which the order kernel would have put in the descriptor.
            const unsigned cnt = p.bin_counts[t], large = p.bin_counts[p.tiles];
            const TileInfo ti = p.tile_info[t];
            unsigned lid[kEmptyTest];  // the large list's first entries (used only when it is that short)
#pragma unroll
            for (int k = 0; k < kEmptyTest; ++k) {
                lid[k] = p.large_list[k];
            }
            const bool bins_invalid = p.fused != 0u && *p.range_tag == p.gen;  // (WorkOrderKernel)
            full = ti.usable == 0u || cnt > p.bin_capacity || bins_invalid;
            flags = (full ? kItemFull : 0u) | (ti.regular != 0u ? kItemRegular : 0u);
            ox = ti.ox;
            oy = ti.oy;
            c_t = full ? 0u : cnt + large;
            list_len = full ? 0u : cnt;
            if (!full && cnt == 0u && large <= static_cast<unsigned>(kEmptyTest) && nchunks == 1u) {
                const Box tb{ti.box.x, ti.box.y, ti.box.z, ti.box.w};  // the empty test (WorkOrderKernel)
                CullRecord lr[kEmptyTest];
#pragma unroll
                for (int k = 0; k < kEmptyTest; ++k) {
                    if (static_cast<unsigned>(k) < large) {
                        lr[k] = p.cull[lid[k]];
                    }
                }
                bool may = false;
#pragma unroll
                for (int k = 0; k < kEmptyTest; ++k) {
                    if (static_cast<unsigned>(k) < large) {
                        const Record q{lr[k].a.x, lr[k].a.y, lr[k].a.z, lr[k].a.w, lr[k].b.x, lr[k].b.y, lr[k].b.z,
                                       lr[k].b.w, lr[k].x.x};
                        may = may || (ScreenBoxOverlaps(tb, lr[k].sb) && BoxMayHit(tb, q));
                    }
                }
                flags |= may ? 0u : kItemEmpty;
            }
        } else {
            flags = w0.w;
            ox = __uint_as_float(w1.x);
            oy = __uint_as_float(w1.y);
            full = (flags & kItemFull) != 0u;
            c_t = full ? 0u : w0.y;
            list_len = full ? 0u : w0.z;
        }
        // A FULL tile streams every record in its part's first chunk; the plan's other chunks of
        // the part (the plan is made as if the bins were valid) have no candidates and publish misses.
        src.full = full && chunk == 0u;
        if (!src.full) {
            // candidates cut into n chunks: chunk c = [c q + c r / n, (c + 1) q + (c + 1) r / n), q r = c_t / n, % n
            const unsigned q = c_t / nchunks, r = c_t % nchunks;
            src.list = p.bin_lists + static_cast<size_t>(t) * p.bin_capacity;
            src.list2 = p.large_list;
            src.count1 = list_len;
            src.begin = chunk * q + chunk * r / nchunks;
            src.end = (chunk + 1u) * q + (chunk + 1u) * r / nchunks;
        }
    } else {
        item = blockIdx.y * gridDim.x + blockIdx.x;
    }
    const unsigned tile = item / kParts;
    const int tx = static_cast<int>(tile % static_cast<unsigned>(p.tiles_x));
    const int ty = static_cast<int>(tile / static_cast<unsigned>(p.tiles_x));
    const int row0 = ty * kTileRows + static_cast<int>(item % kParts) * kBlockRows;  // band row of the block
    if (row0 >= p.row_count) {
        return;  // the last tile row's empty part
    }
    if (p.out_packed != nullptr && threadIdx.x == 0 && chunk == 0u && item % kParts == 0u) {
        // The tile's sample offset in the packed ids when every ray of the tile has it (the deferred
        // shading then reads no per-pixel offsets for the tile), else NaNs (render.h PackedIds).
        const float qn = __builtin_nanf("");
        *reinterpret_cast<float2*>(PackedTileOffset(p.out_packed, p, ty * kTileRows, tx)) =
            (flags & kItemRegular) != 0u ? make_float2(ox, oy) : make_float2(qn, qn);
    }
    const int tid = threadIdx.x;
    const int lane = tid & (kWave - 1);
    const int wave = __builtin_amdgcn_readfirstlane(tid / kWave);
    if (flags & kItemEmpty) {  // every pixel misses (BuildWorkOrder): the miss value, no rays
        const int xe = tx * kWave + lane;
        if (p.out_packed != nullptr) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int y = row0 + wave * R + r;
                if (y < p.row_count) {
                    StorePackedIds(p, tx, xe, y, -1);
                }
            }
        } else if (xe < p.width) {
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const int y = row0 + wave * R + r;
                if (y < p.row_count) {
                    StorePixel(p, xe, y, 0.f, 0.f, -1);
                }
            }
        }
        SRT_DIAG_END(item, chunk, nchunks, 1u, src.full);
        return;
    }
    // LIST: the first batch's records are requested before the rays are set up (its loads
    // are the block's longest dependency chain: list entry, then the 64-B record).
    const unsigned total = src.end - src.begin;
    typename Recs::Raw nxt[kSlices];
    // The list entries run one batch ahead of the records: batch b's prefetch loads batch b + 1's
    // records from entries that arrived during batch b - 1's walk, then requests batch b + 2's
    // entries (one load chain per batch no longer waits in front of the walk).
    unsigned nid[kSlices];
    auto load_ids = [&](unsigned b0) {
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            const unsigned v = b0 + e * kCullThreads + tid;
            if (InBatch(e, tid)) {
                const unsigned vv = src.begin + (v < total ? v : 0u);
                nid[e] = vv < src.count1 ? src.list[vv] : src.list2[vv - src.count1];
            }
        }
    };
    auto load_recs = [&] {
#pragma unroll
        for (int e = 0; e < kSlices; ++e) {
            if (InBatch(e, tid)) {
                nxt[e] = Recs::Load(p, nid[e]);
            }
        }
    };
    auto load_list = [&](unsigned b0) {  // b0: the batch whose records are loaded now
        load_recs();
        if (b0 + kPacketBatch < total) {
            load_ids(b0 + kPacketBatch);
        }
    };
    if (!src.full && total != 0u) {
        load_ids(0u);
        load_list(0u);
    }
    // Rays: lane = column x; rows y0 .. y0 + R - 1. A regular tile (every ray with the sample
    // offset (ox, oy)) computes them without reading the offsets: fx per lane, and row r's fy
    // from lane (wave R + r) of fy_lane (the GenerateRays expressions, bit for bit).
    const int x = tx * kWave + lane;
    const int y0 = row0 + wave * R;
    const bool regular = (flags & kItemRegular) != 0u;
    float fy_lane = __builtin_nanf("");
    Rays<R> s;
    Box lane_box;
    if (regular) {
        if (lane < kBlockRows) {
            const int yc = min(row0 + lane, p.row_count - 1);
            fy_lane = (static_cast<float>(FrameRow(p.row_begin, p.row_interleave, yc)) + oy) / p.hf;
        }
        const int xc = min(x, p.width - 1);
        const float fx = (static_cast<float>(xc) + ox) / p.wf;
        lane_box = Box{fx, fx, __builtin_inff(), -__builtin_inff()};
#pragma unroll
        for (int r = 0; r < R; ++r) {
            s.fx[r] = fx;
            s.fy[r] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(fy_lane), wave * R + r));
            lane_box.ylo = fminf(lane_box.ylo, s.fy[r]);
            lane_box.yhi = fmaxf(lane_box.yhi, s.fy[r]);
        }
        lane_box.xlo = fx != fx ? __builtin_inff() : fx;  // NaN positions drop out of the box
        lane_box.xhi = fx != fx ? -__builtin_inff() : fx;
    } else {
        GenerateRays<R>(p, x, y0, s, lane_box);
    }
    const Box wb = WaveReduceBox(lane_box);
    if (lane == 0) {
        sh.wave_box[wave] = wb;
    }
    __syncthreads();
    Box bb = sh.wave_box[0];  // the block's ray box
#pragma unroll
    for (int w = 1; w < kCullWaves; ++w) {
        const Box o = sh.wave_box[w];
        bb = Box{fminf(bb.xlo, o.xlo), fmaxf(bb.xhi, o.xhi), fminf(bb.ylo, o.ylo), fmaxf(bb.yhi, o.yhi)};
    }
    const int nc = min(kWave, p.width - tx * kWave), nr = min(kBlockRows, p.row_count - row0);
    PacketTables(sh, s, regular, s.fx[0], fy_lane, nc, nr);
    for (int i = tid; i < kBlockRows * kWave; i += kCullThreads) {
        (&sh.keys[0][0])[i] = ~0ull;
    }
    for (int i = tid; i < 2 * kWindowPackets; i += kCullThreads) {
        (&sh.pk[0][0])[i] = make_uint2(0u, 0u);
    }
    unsigned pk_buf = 0u;  // range-end bitmap buffer of the next batch
    const PacketFrame pf = MakePacketFrame(sh, nc, nr, ScreenBoxUsable(bb));
    __syncthreads();  // keys initialised
#ifdef SRT_DIAG
    {
        const unsigned long long now = __builtin_amdgcn_s_memtime();
        d_gather += now - d_mark;
        d_mark = now;
    }
#endif
    if (!src.full) {
        // LIST: candidates [begin, end) of the tile's virtual list, one batch ahead.
#pragma unroll 1
        for (unsigned b0 = 0; b0 < total; b0 += kPacketBatch) {
            CullRecord cr[kSlices];
            bool valid[kSlices];
#pragma unroll
            for (int e = 0; e < kSlices; ++e) {
                cr[e] = Recs::Make(p, nxt[e]);
                valid[e] = InBatch(e, tid) && b0 + e * kCullThreads + tid < total;
            }
            PacketBatch(sh, bb, pf, cr, valid, pk_buf, [&] {
                if (b0 + kPacketBatch < total) {
                    load_list(b0 + kPacketBatch);
                }
            });
            pk_buf ^= 1u;
#ifdef SRT_DIAG
            ++d_batches;
#endif
        }
#ifdef SRT_DIAG
        d_cand = total;
#endif
    } else {
        // FULL: stream every record's quantized screen box in spatial order (one per thread per
        // step, loaded one step ahead); the positions overlapping the block box join an LDS list,
        // walked in packet batches (cull records by position) whenever it holds a batch (and at
        // the end).
        const bool block_sb = pf.use_sb;
        const QBox bq = Quantize(bb);
        const unsigned long long lt_mask = (1ull << lane) - 1ull;
        const unsigned nsteps = p.n_pad / kStreamStep;
        uint2 nq = p.qboxes[tid];
        unsigned listed = 0u;  // ids in the list (block-uniform)
#pragma unroll 1
        for (unsigned k = 0; k < nsteps; ++k) {
            const uint2 q = nq;
            if (k + 1 < nsteps) {
                nq = p.qboxes[(k + 1) * kStreamStep + tid];
            }
            // Disabled records carry empty boxes; unbounded ones span the int16 range.
            const bool pass = !block_sb || QBoxOverlaps(bq, q.x, q.y);
            const unsigned long long m = __ballot(pass);
            const unsigned ph = k & 1u;
            if (lane == 0) {
                sh.counts[ph][wave] = __popcll(m);
            }
            __syncthreads();
            unsigned off = listed, step_n = 0u;
#pragma unroll
            for (int w = 0; w < kCullWaves; ++w) {
                const unsigned cw = sh.counts[ph][w];
                off += w < wave ? cw : 0u;
                step_n += cw;
            }
            if (pass) {
                sh.ids[off + __popcll(m & lt_mask)] = k * kStreamStep + tid;
            }
            listed += step_n;
            if (listed < kPacketBatch && k + 1 < nsteps) {  // block-uniform
                continue;
            }
            __syncthreads();  // every wave's ids are in the list
            // The list shares LDS with the survivor planes: every id this thread walks is read
            // into registers before the first batch writes them.
            unsigned my_ids[kFlushBatches][kSlices];
#pragma unroll
            for (int bi = 0; bi < kFlushBatches; ++bi) {
#pragma unroll
                for (int e = 0; e < kSlices; ++e) {
                    const unsigned v = bi * kPacketBatch + e * kCullThreads + tid;
                    my_ids[bi][e] = InBatch(e, tid) && v < listed ? sh.ids[v] : 0u;
                }
            }
#pragma unroll
            for (int bi = 0; bi < kFlushBatches; ++bi) {
                const unsigned b0 = bi * kPacketBatch;
                if (b0 >= listed) {  // block-uniform
                    break;
                }
                CullRecord cr[kSlices];
                bool valid[kSlices];
#pragma unroll
                for (int e = 0; e < kSlices; ++e) {
                    valid[e] = InBatch(e, tid) && b0 + e * kCullThreads + tid < listed;
                    cr[e] = Recs::Make(p, Recs::Load(p, my_ids[bi][e]));
                }
                PacketBatch(sh, bb, pf, cr, valid, pk_buf, [] {});
                pk_buf ^= 1u;
#ifdef SRT_DIAG
                ++d_batches;
                d_cand += min(listed - b0, static_cast<unsigned>(kPacketBatch));
#endif
            }
            listed = 0u;
        }
    }
    __syncthreads();  // every wave's walk has merged its hits into sh.keys
#ifdef SRT_DIAG
    d_walk = __builtin_amdgcn_s_memtime() - d_mark;
#endif
    unsigned long long key[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
        key[r] = sh.keys[wave * R + r][lane];
    }
    if (nchunks > 1u) {
        constexpr int kPix = kBlockRows * kWave;
        unsigned long long* slices = p.split_keys + static_cast<size_t>(slot) * kPix;
        const int pix = wave * R * kWave + lane;
        [[maybe_unused]] auto publish = [&] {  // this chunk's keys, write-through (sc1) stores, complete before the barrier
#pragma unroll
            for (int r = 0; r < R; ++r) {
                __hip_atomic_store(slices + static_cast<size_t>(chunk) * kPix + pix + r * kWave, key[r],
                                   __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        };
        // Split part: publish this chunk's keys, count the arrival; the last of the part's chunks
        // takes the minimum over every chunk's keys (sc1 loads) and shades. Hand-off form:
        // MI355X_MICROARCH.md "Valid forms", table row 1 (sc1 stores, every storing wave's
        // vmcnt(0), barrier, one agent-scope add; the last adder's block loads sc1 after a barrier).
        publish();
        if (tid == 0) {
            const unsigned before = __hip_atomic_fetch_add(&p.arrive[slot], 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const unsigned last = before == nchunks - 1u ? 1u : 0u;
            if (last != 0u) {  // every chunk has arrived: reset for the next frame
                __hip_atomic_store(&p.arrive[slot], 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            sh.last = last;
        }
        __syncthreads();
        if (sh.last == 0u) {
            SRT_DIAG_END(item, chunk, nchunks, 0u, src.full);
            return;
        }
        for (unsigned c = 0; c < nchunks; ++c) {
            if (c == chunk) {
                continue;
            }
#pragma unroll
            for (int r = 0; r < R; ++r) {
                const unsigned long long o = __hip_atomic_load(slices + static_cast<size_t>(c) * kPix + pix + r * kWave,
                                                               __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
                key[r] = o < key[r] ? o : key[r];
            }
        }
    }
    if (p.out_packed != nullptr) {  // packed ids: every lane of the wave takes part (ballots)
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int y = y0 + r;
            if (y < p.row_count) {
                StorePackedIds(p, tx, x, y, key[r] != ~0ull ? static_cast<int>(static_cast<unsigned>(key[r])) : -1);
            }
        }
    } else if (x < p.width && p.out_ids != nullptr) {
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int y = y0 + r;
            if (y < p.row_count) {
                StorePixel(p, x, y, 0.f, 0.f, key[r] != ~0ull ? static_cast<int>(static_cast<unsigned>(key[r])) : -1);
            }
        }
    } else if (x < p.width) {
        // RGBA: every row's shading record is loaded before any is used (a miss loads triangle 0's,
        // unused), so the rows' loads share one round trip; per row in a branch they took one each,
        // at the end of every block.
        int id[R];
        float4 nr[R], al[R];
#pragma unroll
        for (int r = 0; r < R; ++r) {
            id[r] = key[r] != ~0ull ? static_cast<int>(static_cast<unsigned>(key[r])) : -1;
            const float4* sr = p.shade + 2ull * static_cast<unsigned>(max(id[r], 0));
            nr[r] = sr[0];
            al[r] = sr[1];
        }
#pragma unroll
        for (int r = 0; r < R; ++r) {
            const int y = y0 + r;
            if (y < p.row_count) {
                const float2 f = sh.fxy[wave * R + r][lane];
                StoreRgba(p, x, y, ShadeRecord(p, f.x, f.y, id[r], nr[r], al[r]));
            }
        }
    }
    SRT_DIAG_END(item, chunk, nchunks, 1u, src.full);
#undef SRT_DIAG_END
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

// Smallest candidate chunk of a split tile part; env SRT_CULL_CHUNK, a multiple of 64 (default
// 256: one packet-walk batch).
unsigned CullChunkFromEnv() {
    const char* v = std::getenv("SRT_CULL_CHUNK");
    const long c = v == nullptr || *v == '\0' ? 256 : std::strtol(v, nullptr, 10);
    return c < 64 ? 64u : static_cast<unsigned>((c + 63) / 64 * 64);
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
void LaunchLds(K kernel, dim3 grid, dim3 block, std::size_t lds, hipStream_t stream, hipEvent_t start, hipEvent_t stop,
               const P& p) {
    if (start != nullptr || stop != nullptr) {
        hipExtLaunchKernelGGL(kernel, grid, block, lds, stream, start, stop, 0, p);
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, stream, p);
    }
}
template <class K, class P>
void Launch(K kernel, dim3 grid, dim3 block, hipStream_t stream, hipEvent_t start, hipEvent_t stop, const P& p) {
    LaunchLds(kernel, grid, block, 0, stream, start, stop, p);
}

}  // namespace

#ifdef SRT_DIAG
hipError_t DiagRead(void* host, std::size_t bytes) {
    return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_srt_diag), bytes < sizeof(g_srt_diag) ? bytes : sizeof(g_srt_diag));
}
#endif

namespace {
// Carve-up of a scene's edge allocation (render.h kEdgeFloatsPerTriangle): tile-planar edge
// records, screen boxes, quantized boxes, cull records, shading normals.
struct EdgeLayout {
    float4* tiles;
    float4* screen_boxes;
    uint2* qboxes;
    CullRecord* cull;
};
EdgeLayout EdgeBuffers(const float* d_edges, std::uint64_t n) {
    EdgeLayout e;
    const std::uint64_t n_pad = PaddedTriangleCount(n);
    e.tiles = reinterpret_cast<float4*>(const_cast<float*>(d_edges));
    e.screen_boxes = e.tiles + n_pad / kTileTriangles * kTileFloat4;
    e.qboxes = reinterpret_cast<uint2*>(e.screen_boxes + n_pad);
    e.cull = reinterpret_cast<CullRecord*>(e.qboxes + n_pad);
    return e;
}
}  // namespace

namespace {
PrepareParams MakePrepareParams(const float* d_vertices, const unsigned* d_rank, std::uint64_t n, const Frame& frame,
                                float* d_edges) {
    PrepareParams p{};
    p.vertices = d_vertices;
    p.rank = d_rank;
    const EdgeLayout e = EdgeBuffers(d_edges, n);
    p.edges = e.tiles;
    p.screen_boxes = e.screen_boxes;
    p.qboxes = e.qboxes;
    p.cull = e.cull;
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
// Resident trace blocks of the current device (all CUs x blocks per CU), queried once per device.
unsigned TraceSlots() {
    static thread_local int cached_device = -1;
    static thread_local unsigned slots = 0;
    int dev = 0;
    if (hipGetDevice(&dev) == hipSuccess && dev != cached_device) {
        int per_cu = 0, cus = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, TraceCullKernel<TraceBatch>, kCullThreads, 0) == hipSuccess &&
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess) {
            slots = static_cast<unsigned>(per_cu * cus);
            cached_device = dev;
        }
    }
    return slots;
}

long EnvLong(const char* name, long fallback) {
    const char* v = std::getenv(name);
    return v == nullptr || *v == '\0' ? fallback : std::strtol(v, nullptr, 10);
}

// When a cull launch runs the work order (env SRT_WORK_PLAN): "auto" (default) for launches of
// several frames, which fill the chip -- there the order launch overlaps other queues' work, while
// a plan-only trace's extra dependent loads at each block's start cost throughput -- and the slot's
// plan for single-frame launches, whose latency the order launch would lengthen; "reuse": plans
// whenever the slots have one; "order": every launch (a slot without a plan for its trace grid
// always gets the order launch).
enum class WorkPlan { kAuto, kReuse, kOrder };
WorkPlan WorkPlanFromEnv() {
    const char* v = std::getenv("SRT_WORK_PLAN");
    const std::string m = v == nullptr ? "" : v;
    return m == "reuse" ? WorkPlan::kReuse : m == "order" ? WorkPlan::kOrder : WorkPlan::kAuto;
}

struct BinSizes {
    std::size_t info, counts, lists, large, work, work_count, arrive, split_keys, range_tag;
};
BinSizes CullBinSizes(std::uint64_t n, std::size_t width, std::size_t row_count) {
    const std::size_t tx = (width + kWave - 1) / kWave, ty = (row_count + kTileRows - 1) / kTileRows;
    const std::size_t tiles = tx * ty;
    const auto al = [](std::size_t b) { return (b + 255) / 256 * 256; };
    const std::size_t descs = CullDescriptors(tiles, 1);  // the most a launch of this shape lists
    const bool split = descs > tiles * kParts;
    BinSizes z;
    z.info = al(tiles * sizeof(TileInfo));
    z.counts = al(2 * (tiles + 1) * 4);  // two buffers: a frame bins into one, its trace resets the other
    z.lists = al(tiles * static_cast<std::size_t>(CullBinCapacity(n, tiles)) * 4);
    z.large = al(PaddedTriangleCount(n) * 4);
    z.work = al(descs * 2 * sizeof(uint4));
    z.work_count = al(kOrderWords * 4);
    z.arrive = split ? al(descs * 4) : 0;
    z.split_keys = split ? al(descs * kBlockRows * kWave * 8) : 0;
    z.range_tag = al(4);
    return z;
}
}  // namespace

unsigned CullDescriptors(std::size_t tiles, std::size_t frames) {
    const std::size_t parts = tiles * kParts;
    frames = frames == 0 ? 1 : frames;
    const long forced = EnvLong("SRT_CULL_CHUNKS", 0);
    if (forced > 0) {  // measurement / tests: room for `forced` descriptors per part
        return static_cast<unsigned>(parts * static_cast<std::size_t>(forced < kMaxChunks ? forced : kMaxChunks));
    }
    const std::size_t slots = TraceSlots();
    // Parts that leave the chip partly idle (small bands): M = ceil(slots / all parts) each.
    std::size_t m = parts * frames >= slots || parts == 0 ? 1 : (slots + parts * frames - 1) / (parts * frames);
    m = m < static_cast<std::size_t>(kMaxChunks) ? m : kMaxChunks;
    // Room to cut the heavy parts: SRT_CULL_SPLIT extra descriptors per launch (default: one per
    // resident block), shared by the launch's frames.
    const long extra = EnvLong("SRT_CULL_SPLIT", static_cast<long>(slots));
    const std::size_t e = extra > 0 ? static_cast<std::size_t>(extra) / frames : 0;
    const std::size_t d = parts * m > parts + e ? parts * m : parts + e;
    return static_cast<unsigned>(d);
}

std::size_t CullBinBytes(std::uint64_t n, std::size_t width, std::size_t row_count) {
    const BinSizes z = CullBinSizes(n, width, row_count);
    return z.info + z.counts + z.lists + z.large + z.work + z.work_count + z.arrive + z.split_keys + z.range_tag;
}

std::size_t CullBinCounterBytes(std::uint64_t n, std::size_t width, std::size_t row_count) {
    const BinSizes z = CullBinSizes(n, width, row_count);
    return z.counts + z.work_count + z.arrive + z.range_tag;
}

CullBins CullBinLayout(void* base, std::uint64_t n, std::size_t width, std::size_t row_count, unsigned parity) {
    const BinSizes z = CullBinSizes(n, width, row_count);
    unsigned char* w = static_cast<unsigned char*>(base);
    CullBins b{};
    auto take = [&w](std::size_t bytes) {
        unsigned char* at = w;
        w += bytes;
        return at;
    };
    // The counters first (CullBinCounterBytes: the only bytes that must start zero), then the buffers
    // every frame writes before it reads them.
    unsigned* counts = reinterpret_cast<unsigned*>(take(z.counts));
    b.work_count = reinterpret_cast<unsigned*>(take(z.work_count));
    b.arrive = reinterpret_cast<unsigned*>(take(z.arrive));
    b.range_tag = reinterpret_cast<unsigned*>(take(z.range_tag));
    b.tile_info = take(z.info);
    b.lists = reinterpret_cast<unsigned*>(take(z.lists));
    b.large_list = reinterpret_cast<unsigned*>(take(z.large));
    b.work = take(z.work);
    b.split_keys = take(z.split_keys);
    b.tiles = CullTiles(width, row_count);
    b.counts = counts + (parity & 1u) * (b.tiles + 1);
    b.counts_next = counts + ((parity & 1u) ^ 1u) * (b.tiles + 1);
    b.capacity = CullBinCapacity(n, b.tiles);
    b.descs = z.split_keys != 0 ? CullDescriptors(b.tiles, 1) : static_cast<unsigned>(b.tiles * kParts);
    return b;
}

namespace {
TraceParams MakeTraceParams(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_shade,
                            const Frame& frame, const float background[3], const BandArgs& band) {
    TraceParams p{};
    const EdgeLayout e = EdgeBuffers(d_edges, n);
    p.edges = e.tiles;
    p.screen_boxes = e.screen_boxes;
    p.qboxes = e.qboxes;
    p.cull = e.cull;
    p.vertices = d_vertices;
    p.shade = reinterpret_cast<const float4*>(d_shade);
    p.offsets = reinterpret_cast<const float2*>(band.offsets);
    p.out = reinterpret_cast<float4*>(band.rgba);
    const bool packed = band.id_planes >= 0 && band.ids != nullptr;
    p.out_ids = packed ? nullptr : band.ids;
    p.out_packed = packed ? reinterpret_cast<unsigned char*>(band.ids) : nullptr;
    if (packed) {
        const PackedIds lay = PackedIdLayout(band.id_planes, band.row_count, band.width);
        p.id_planes = band.id_planes;
        p.id_words = static_cast<unsigned>(lay.words);
        p.id_low_row_bytes = static_cast<unsigned>(lay.low_row_bytes);
        p.id_row_bytes = static_cast<unsigned>(lay.row_bytes);
        p.id_tile_row_bytes = static_cast<unsigned>(lay.tile_row_bytes);
    }
    p.out_frame_rows = band.rgba_frame_rows ? 1 : 0;
    p.n_pad = static_cast<unsigned>(PaddedTriangleCount(n));
    p.n_tiles = static_cast<unsigned>(n == 0 ? 1 : (n + kTileTriangles - 1) / kTileTriangles);
    p.width = static_cast<int>(band.width);
    p.row_count = static_cast<int>(band.row_count);
    p.row_begin = static_cast<int>(band.row_begin);
    p.row_interleave = static_cast<int>(band.row_interleave);
    p.wf = static_cast<float>(band.width);
    p.hf = static_cast<float>(band.height);
    for (int k = 0; k < 3; ++k) {
        p.base[k] = frame.base[k];
        p.du[k] = frame.du[k];
        p.dv[k] = frame.dv[k];
        p.bg[k] = background[k];
        p.eye[k] = frame.origin[k];
    }
    p.n = static_cast<unsigned>(n);
    p.tiles_x = static_cast<int>((band.width + kWave - 1) / kWave);
    p.tiles = static_cast<unsigned>(p.tiles_x) * static_cast<unsigned>((band.row_count + kTileRows - 1) / kTileRows);
#ifdef SRT_DIAG
    if (const char* x = std::getenv("SRT_EXP")) {
        p.exp = static_cast<unsigned>(std::strtoul(x, nullptr, 0));
    }
#endif
    return p;
}

// The bin stage's parameters for trace parameters `p` and its bins; binds the bins to `p`.
BinParams BindBins(TraceParams& p, const CullBins& bins, std::uint64_t n) {
    BinParams b{};
    b.offsets = p.offsets;
    b.cull = p.cull;
    b.tile_info = static_cast<TileInfo*>(bins.tile_info);
    b.counts = bins.counts;
    b.lists = bins.lists;
    b.large_list = bins.large_list;
    b.work = static_cast<uint4*>(bins.work);
    b.work_count = bins.work_count;
    b.range_tag = bins.range_tag;
    b.gen = bins.gen;
    b.capacity = bins.capacity;
    b.descs = bins.descs;
    b.min_chunk = CullChunkFromEnv();
    b.n = static_cast<unsigned>(n);
    b.tiles_x = p.tiles_x;
    b.tiles_y = static_cast<int>(p.tiles / static_cast<unsigned>(p.tiles_x));
    b.width = p.width;
    b.row_count = p.row_count;
    b.row_begin = p.row_begin;
    b.row_interleave = p.row_interleave;
    b.wf = p.wf;
    b.hf = p.hf;
    b.exp = p.exp;
    p.tile_info = b.tile_info;
    p.order = bins.order;
    p.svertices = bins.svertices;
    p.work = b.work;
    p.work_count = b.work_count;
    p.split_keys = static_cast<unsigned long long*>(bins.split_keys);
    p.arrive = bins.arrive;
    p.bin_lists = bins.lists;
    p.bin_counts = bins.counts;
    p.bin_counts_next = bins.counts_next;
    p.range_tag = bins.range_tag;
    p.gen = bins.gen;
    p.large_list = bins.large_list;
    p.bin_capacity = bins.capacity;
    return b;
}
}  // namespace

namespace {
// The four stage launches of a batched cull frame set; TB / BB / PB: the frames' parameters as
// kernel arguments (FrameArgs) or a device table (FrameTable).
template <class TB, class BB, class PB>
void LaunchCullStages(const TB& tb, const BB& bb, const PB& pb, unsigned z, unsigned gx, unsigned gy, unsigned blocks,
                      bool fused, bool order, bool recompute, unsigned descs, hipStream_t stream,
                      const StageEvents& ev) {
    if (!fused) {
        Launch(TileInfoKernel<BB>, dim3(gx, (gy + kInfoTiles - 1) / kInfoTiles, z), dim3(kBinThreads), stream,
               ev.prep_begin, ev.prep_end, bb);
    }
    if (fused) {
        LaunchLds(PrepareBinKernel<PB, false>, dim3(blocks, 1, z), dim3(kBinThreads),
                  BinLdsBytes(static_cast<int>(gx), static_cast<int>(gy)), stream, ev.bin_begin,
                  order ? nullptr : ev.bin_end, pb);
    } else {
        LaunchLds(PrepareBinKernel<PB, true>, dim3(blocks, 1, z), dim3(kBinThreads),
                  BinLdsBytes(static_cast<int>(gx), static_cast<int>(gy)), stream, ev.bin_begin,
                  order ? nullptr : ev.bin_end, pb);
    }
    if (!order) {  // the slots' plans are current: the trace follows the bins
        if (recompute) {
            Launch(TraceCullKernel<TB, true>, dim3(descs, 1, z), dim3(kWave * kCullWaves), stream, ev.begin, ev.end, tb);
        } else {
            Launch(TraceCullKernel<TB, false>, dim3(descs, 1, z), dim3(kWave * kCullWaves), stream, ev.begin, ev.end, tb);
        }
        return;
    }
    LaunchLds(WorkOrderKernel<BB>, dim3((gx * gy + kOrderBlock - 1) / kOrderBlock, 1, z), dim3(kOrderBlock),
              OrderLdsBytes(static_cast<int>(gx * gy)), stream, nullptr, ev.bin_end, bb);
    if (recompute) {
        Launch(TraceCullKernel<TB, true>, dim3(descs, 1, z), dim3(kWave * kCullWaves), stream, ev.begin, ev.end, tb);
    } else {
        Launch(TraceCullKernel<TB, false>, dim3(descs, 1, z), dim3(kWave * kCullWaves), stream, ev.begin, ev.end, tb);
    }
}

// Layout of a parameter table (CullTableBytes): PrepareBinParams, BinParams, TraceParams arrays.
struct TableLayout {
    std::size_t prep, bin, trace, bytes;
};
TableLayout MakeTableLayout(std::size_t frames) {
    const auto al = [](std::size_t b) { return (b + 255) / 256 * 256; };
    TableLayout t;
    t.prep = 0;
    t.bin = al(frames * sizeof(PrepareBinParams));
    t.trace = t.bin + al(frames * sizeof(BinParams));
    t.bytes = t.trace + al(frames * sizeof(TraceParams));
    return t;
}
}  // namespace

std::size_t CullTableBytes(std::size_t frames) { return MakeTableLayout(frames).bytes; }

// The parameter table's upload: one 16-B word per thread, read from page-locked host memory over the
// bus (one round trip for the whole table) and stored to the device table.
__global__ __launch_bounds__(256) void UploadTableKernel(const uint4* __restrict__ host, uint4* __restrict__ dev,
                                                         size_t n16) {
    const size_t i = static_cast<size_t>(blockIdx.x) * 256 + threadIdx.x;
    if (i < n16) {
        dev[i] = host[i];
    }
}

hipError_t LaunchCullFrames(const CullFrame* frames, std::size_t count, std::uint64_t n, const float* d_vertices,
                            const float* d_shade, const Frame& frame, const float background[3], const unsigned* d_rank,
                            hipStream_t stream, const StageEvents* events, const CullTable* table) {
    const bool use_table = count > static_cast<std::size_t>(kMaxBatch);
    if (frames == nullptr || count == 0 || count > static_cast<std::size_t>(kMaxTableFrames) ||
        (use_table && (table == nullptr || table->device == nullptr || table->host == nullptr ||
                       count > table->frames))) {
        return hipErrorInvalidValue;
    }
    const BandArgs& band0 = frames[0].band;
    if (band0.row_count == 0 || band0.width == 0) {
        return hipSuccess;
    }
    if (!CullBinnable(band0.width, band0.row_count)) {
        return hipErrorInvalidValue;
    }
    const StageEvents ev = events != nullptr ? *events : StageEvents{};
    TraceBatch tb{};
    BinBatch bb{};
    PrepareBinBatch pb{};
    const TableLayout lay = MakeTableLayout(count);
    unsigned char* host = use_table ? static_cast<unsigned char*>(table->host) : nullptr;
    PrepareBinParams* pp = use_table ? reinterpret_cast<PrepareBinParams*>(host + lay.prep) : pb.f;
    BinParams* bp = use_table ? reinterpret_cast<BinParams*>(host + lay.bin) : bb.f;
    TraceParams* tp = use_table ? reinterpret_cast<TraceParams*>(host + lay.trace) : tb.f;
    // Fused tile info only when every frame of the launch has the band's shape AND its first row
    // (per-frame bands -- share senders, rotated bands -- always compute their tile info first).
    bool fused = CullFusedInfo(band0.row_begin, band0.row_count, band0.height, band0.row_interleave);
    for (std::size_t i = 1; i < count && fused; ++i) {
        fused = frames[i].band.row_begin == band0.row_begin;
    }
    bool order = false;  // some frame's slot needs its work plan (re)built: the order launch runs for all
    for (std::size_t i = 0; i < count; ++i) {
        const CullFrame& f = frames[i];
        if (f.bins == nullptr || f.edges == nullptr || f.bins->order == nullptr || f.bins->svertices == nullptr ||
            f.band.width != band0.width ||
            f.band.row_count != band0.row_count || (fused && f.band.row_begin != band0.row_begin) ||
            f.band.row_interleave != band0.row_interleave ||
            f.band.height != band0.height || f.bins->descs != frames[0].bins->descs ||
            f.bins->recompute != frames[0].bins->recompute) {
            return hipErrorInvalidValue;  // one band shape per batch (its first row may differ per frame)
        }
        tp[i] = MakeTraceParams(f.edges, n, d_vertices, d_shade, frame, background, f.band);
        if (f.bins->tiles != tp[i].tiles) {
            return hipErrorInvalidValue;  // bins sized for another band shape
        }
        bp[i] = BindBins(tp[i], *f.bins, n);
        bp[i].fused = fused ? 1u : 0u;
        bp[i].recompute = f.bins->recompute ? 1u : 0u;
        tp[i].fused = bp[i].fused;
        order = order || f.bins->plan;
        pp[i].prep = MakePrepareParams(d_vertices, d_rank, n, frame, const_cast<float*>(f.edges));
        pp[i].prep.order = f.bins->order;
        pp[i].prep.svertices = f.bins->svertices;
        pp[i].prep.block_ext = f.bins->block_ext;
        pp[i].bin = bp[i];
    }
    static const WorkPlan plan_mode = WorkPlanFromEnv();
    order = order || plan_mode == WorkPlan::kOrder || (plan_mode == WorkPlan::kAuto && count > 1);
    for (std::size_t i = 0; i < count; ++i) {
        tp[i].plan_only = order ? 0u : 1u;
    }
    const unsigned z = static_cast<unsigned>(count);
    const unsigned gx = static_cast<unsigned>(tp[0].tiles_x), gy = tp[0].tiles / gx;
    const unsigned info_blocks = gx * ((gy + kInfoTiles - 1) / kInfoTiles);
    // Tile info (fused: extra blocks of the bin launch); records + bins (every padded position: the
    // FULL stream reads them all); the trace work list; the trace: one block per work descriptor
    // (grid z = frame; interleaving the frames' descriptors so every frame's heaviest work starts
    // first measured no faster).
    const unsigned blocks = (pp[0].prep.n_pad + kBinThreads - 1) / kBinThreads + (fused ? info_blocks : 0u);
    const unsigned descs = frames[0].bins->descs;
    if (!use_table) {
        LaunchCullStages(tb, bb, pb, z, gx, gy, blocks, fused, order, frames[0].bins->recompute, descs, stream, ev);
        return hipGetLastError();
    }
    // One upload of every frame's parameters, then the same four launches reading them from it.
    if (table->host_device != nullptr) {
        const std::size_t n16 = (lay.bytes + 15) / 16;
        hipLaunchKernelGGL(UploadTableKernel, dim3(static_cast<unsigned>((n16 + 255) / 256)), dim3(256), 0, stream,
                           static_cast<const uint4*>(table->host_device), static_cast<uint4*>(table->device), n16);
    } else {
        const hipError_t e = hipMemcpyAsync(table->device, table->host, lay.bytes, hipMemcpyHostToDevice, stream);
        if (e != hipSuccess) {
            return e;
        }
    }
    if (table->uploaded != nullptr) {
        const hipError_t e = hipEventRecord(table->uploaded, stream);
        if (e != hipSuccess) {
            return e;
        }
    }
    unsigned char* dev = static_cast<unsigned char*>(table->device);
    const PrepareBinTable pt{(ConstantPtr<PrepareBinParams>)(dev + lay.prep)};
    const BinTable bt{(ConstantPtr<BinParams>)(dev + lay.bin)};
    const TraceTable tt{(ConstantPtr<TraceParams>)(dev + lay.trace)};
    LaunchCullStages(tt, bt, pt, z, gx, gy, blocks, fused, order, frames[0].bins->recompute, descs, stream, ev);
    return hipGetLastError();
}

hipError_t LaunchTrace(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_shade,
                       const Frame& frame, const float background[3], const BandArgs& band, int variant,
                       const CullBins* bins, hipStream_t stream, const StageEvents* events,
                       const unsigned* prepare_rank, void* bvh) {
    if (band.row_count == 0 || band.width == 0) {
        return hipSuccess;
    }
    if (variant == kTraceCull && bins != nullptr) {  // computes the records itself, every call
        const CullFrame f{d_edges, bins, band};
        return LaunchCullFrames(&f, 1, n, d_vertices, d_shade, frame, background, nullptr, stream, events, nullptr);
    }
    const StageEvents ev = events != nullptr ? *events : StageEvents{};
    if (prepare_rank != nullptr) {
        const hipError_t e = LaunchPrepare(d_vertices, prepare_rank, n, frame, const_cast<float*>(d_edges), stream,
                                           ev.prep_begin, ev.prep_end);
        if (e != hipSuccess) {
            return e;
        }
    }
    const TraceParams p = MakeTraceParams(d_edges, n, d_vertices, d_shade, frame, background, band);
    const unsigned gx = static_cast<unsigned>(p.tiles_x);
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
    } else if (variant == kTraceScalar) {
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerLane - 1) / kRowsPerLane);
        Launch(TraceScalarKernel, dim3(gx, gy), dim3(kWave), stream, ev.begin, ev.end, p);
    } else if (variant == kTraceCull) {
        // Unbinned: one block per (tile, part), gridDim.x = tile columns, gridDim.y = tile rows x
        // parts; every block streams every record.
        TraceBatch tb{};
        tb.f[0] = p;
        Launch(TraceCullKernel<TraceBatch>, dim3(gx, p.tiles / gx * kParts), dim3(kWave * kCullWaves), stream, ev.begin, ev.end,
               tb);
    } else {
        constexpr int kRowsPerBlock = kRowsPerLane * kLdsWaves;
        const unsigned gy = static_cast<unsigned>((band.row_count + kRowsPerBlock - 1) / kRowsPerBlock);
        Launch(TraceLdsKernel, dim3(gx, gy), dim3(kWave * kLdsWaves), stream, ev.begin, ev.end, p);
    }
    return hipGetLastError();
}

std::size_t BlockExtentCount(std::uint64_t n) {
    return static_cast<std::size_t>((PaddedTriangleCount(n) + kBinThreads - 1) / kBinThreads);
}

hipError_t LaunchBlockExtents(const float* d_svertices, std::uint64_t n, const Frame& frame, float2* d_ext,
                              hipStream_t stream) {
    if (n == 0 || d_svertices == nullptr || d_ext == nullptr) {
        return hipErrorInvalidValue;
    }
    PrepareParams pp = MakePrepareParams(nullptr, nullptr, n, frame, nullptr);
    pp.svertices = d_svertices;
    hipLaunchKernelGGL(BlockExtentKernel, dim3((pp.n_pad + kBinThreads - 1) / kBinThreads), dim3(kBinThreads), 0, stream,
                       pp, d_ext);
    return hipGetLastError();
}

bool CullFusedInfo(std::size_t row_begin, std::size_t row_count, std::size_t height, std::size_t interleave) {
    static const bool enabled = [] {
        const char* v = std::getenv("SRT_FUSED_INFO");
        return v == nullptr || std::strcmp(v, "0") != 0;
    }();
    // Bands of at least SRT_FUSED_BAND_PCT % of the frame's rows too (default 75: the share
    // compositor's own band): their bin launch then writes every cull record, as the tile info it
    // would test them against is not known yet -- nearly all of them are needed anyway. (Every band
    // fused measured slower at every P, the thin ones paying for all records: P = 8 rank 5.35 -> 6.0
    // us, round 4.)
    static const std::size_t band_pct = [] {
        const char* v = std::getenv("SRT_FUSED_BAND_PCT");
        const long n = v != nullptr ? std::strtol(v, nullptr, 10) : 75;
        return static_cast<std::size_t>(n < 0 ? 0 : n);
    }();
    if (!enabled || height == 0) {
        return false;
    }
    if (row_begin == 0 && row_count == height && interleave == 1) {
        return true;
    }
    return band_pct <= 100 && row_count * 100 >= band_pct * height;
}

bool BandFits(std::size_t row_begin, std::size_t row_count, std::size_t interleave, std::size_t height) {
    if (interleave == 0 || row_begin > height) {
        return false;
    }
    if (row_count == 0) {
        return true;
    }
    const std::size_t every = interleave & 0xFFFFu, log2 = interleave >> 16;
    if (every == 0 || log2 > 6 || (std::size_t{1} << log2) > every || (interleave > 1 && row_begin % kCullTileRows != 0)) {
        return false;
    }
    return BandFrameRow(row_begin, interleave, row_count - 1) < height;  // earlier tile rows are full
}

std::size_t PatternBandRows(std::size_t height, std::size_t row_begin, std::size_t pattern) {
    if (pattern <= 1) {
        return row_begin < height ? height - row_begin : 0;
    }
    std::size_t rows = 0;
    for (std::size_t local = 0;; local += kCullTileRows) {
        const std::size_t fr = BandFrameRow(row_begin, pattern, local);
        if (fr >= height) {
            return rows;
        }
        rows += std::min<std::size_t>(kCullTileRows, height - fr);
    }
}

std::size_t InterleavedBandRows(std::size_t height, std::size_t bands, std::size_t band) {
    const std::size_t tiles = (height + kCullTileRows - 1) / kCullTileRows;
    std::size_t rows = 0;
    for (std::size_t t = band; t < tiles; t += bands) {
        rows += std::min<std::size_t>(kCullTileRows, height - t * kCullTileRows);
    }
    return rows;
}

int IdPlanes(std::uint64_t triangles) {
    int bits = 16;
    while (bits < 16 + kMaxIdPlanes && (1ull << bits) - 1ull < triangles) {  // codes 0 .. n - 1, miss = all ones
        ++bits;
    }
    return (1ull << bits) - 1ull >= triangles ? bits - 16 : -1;
}

PackedIds PackedIdLayout(int planes, std::size_t rows, std::size_t width) {
    PackedIds l;
    l.planes = planes < 0 ? 0 : planes;
    l.rows = rows;
    l.width = width;
    l.words = (width + kWave - 1) / kWave;
    l.low_row_bytes = (width * 2 + 7) / 8 * 8;
    l.row_bytes = l.low_row_bytes + static_cast<std::size_t>(l.planes) * l.words * 8;
    l.tile_row_bytes = kCullTileRows * l.row_bytes + l.words * 8;
    l.bytes = ((rows + kCullTileRows - 1) / kCullTileRows * l.tile_row_bytes + 255) / 256 * 256;
    return l;
}

hipError_t LaunchShadeTable(const float* d_vertices, const float* d_albedo, std::uint64_t n, float* d_table,
                            hipStream_t stream) {
    if (n == 0) {
        return hipSuccess;
    }
    hipLaunchKernelGGL(ShadeTableKernel, dim3(static_cast<unsigned>((n + 255) / 256)), dim3(256), 0, stream, d_vertices,
                       d_albedo, static_cast<unsigned>(n), reinterpret_cast<float4*>(d_table));
    return hipGetLastError();
}

// The rows of the shade grid (ShadeRowOf's j): every row of the bands a call stores, for interleaved
// bands rounded up to whole cycles of tile rows (the threads past the frame return).
static std::size_t ShadeRowsLaunched(std::size_t row_count, std::size_t band_rows, std::size_t interleaved,
                                     unsigned skip, std::size_t own, std::size_t first_rows) {
    const bool skips = skip != ~0u && skip >= own;
    if (interleaved != 0) {
        const std::size_t dropped = std::min(own, interleaved) + (skips && skip < interleaved ? 1 : 0);
        const std::size_t stored = interleaved - std::min(dropped, interleaved);
        const std::size_t tile_rows = (row_count + kCullTileRows - 1) / kCullTileRows;
        return (tile_rows + interleaved - 1) / interleaved * stored * kCullTileRows;
    }
    const std::size_t F = first_rows != 0 ? first_rows : band_rows;
    const auto start = [&](std::size_t b) { return std::min(row_count, b == 0 ? 0 : F + (b - 1) * band_rows); };
    const std::size_t own_rows = start(own);
    const std::size_t skip_rows = skips ? std::min(skip == 0 ? F : band_rows, row_count - start(skip)) : 0;
    return row_count - own_rows - skip_rows;
}

hipError_t LaunchShade(const float* d_vertices, const float* d_shade, const float* d_edges, std::uint64_t n,
                       const Frame& frame, const float background[3], const BandArgs& band, hipStream_t stream,
                       std::size_t frames, std::size_t band_rows, std::size_t interleaved,
                       std::size_t offsets_stride, long skip_band, std::size_t own_bands, std::size_t first_rows) {
    if (band.row_count == 0 || band.width == 0 || frames == 0) {
        return hipSuccess;
    }
    if (band_rows == 0) {
        band_rows = band.row_count;
    }
    if (band.ids == nullptr || band.rgba == nullptr || band.offsets == nullptr || frames > 65535 || band.row_count > 65535 ||
        band_rows > band.row_count || first_rows > band.row_count || (first_rows != 0 && interleaved != 0)) {
        return hipErrorInvalidValue;
    }
    TraceParams p{};
    (void)d_edges;
    p.n = static_cast<unsigned>(n);
    p.vertices = d_vertices;
    p.shade = reinterpret_cast<const float4*>(d_shade);
    p.offsets = reinterpret_cast<const float2*>(band.offsets);
    p.out = reinterpret_cast<float4*>(band.rgba);
    p.width = static_cast<int>(band.width);
    p.row_count = static_cast<int>(band.row_count);
    p.row_begin = static_cast<int>(band.row_begin);
    p.row_interleave = static_cast<int>(band.row_interleave);
    p.wf = static_cast<float>(band.width);
    p.hf = static_cast<float>(band.height);
    for (int k = 0; k < 3; ++k) {
        p.base[k] = frame.base[k];
        p.du[k] = frame.du[k];
        p.dv[k] = frame.dv[k];
        p.bg[k] = background[k];
        p.eye[k] = frame.origin[k];
    }
    if (band.id_planes >= 0 && (band.id_planes > kMaxIdPlanes || IdPlanes(n) != band.id_planes)) {
        return hipErrorInvalidValue;
    }
    const unsigned skip = skip_band < 0 ? 0xFFFFFFFFu : static_cast<unsigned>(skip_band);
    const std::size_t stored =
        ShadeRowsLaunched(band.row_count, band_rows, interleaved, skip, own_bands, first_rows);
    if (stored == 0) {
        return hipSuccess;
    }
    const dim3 grid(static_cast<unsigned>((band.width + kShadeThreads - 1) / kShadeThreads),
                    static_cast<unsigned>((stored + kShadeRows - 1) / kShadeRows), static_cast<unsigned>(frames));
    const void* ids = band.ids;
    if (band.id_planes >= 0) {
        const PackedIds lay = PackedIdLayout(band.id_planes, band_rows, band.width);
        p.id_planes = band.id_planes;
        p.id_words = static_cast<unsigned>(lay.words);
        p.id_low_row_bytes = static_cast<unsigned>(lay.low_row_bytes);
        p.id_row_bytes = static_cast<unsigned>(lay.row_bytes);
        p.id_tile_row_bytes = static_cast<unsigned>(lay.tile_row_bytes);
        const auto launch = [&](auto kernel) {
            hipLaunchKernelGGL(kernel, grid, dim3(kShadeThreads), 0, stream, p, ids, static_cast<unsigned>(band_rows),
                               static_cast<unsigned>(frames), static_cast<unsigned>(interleaved), offsets_stride / 2,
                               skip, static_cast<unsigned>(own_bands), lay.bytes, static_cast<unsigned>(first_rows));
        };
        switch (band.id_planes) {  // the bit planes as a template argument: their loads unrolled
            case 0: launch(ShadeIdsKernel<true, 0>); break;
            case 1: launch(ShadeIdsKernel<true, 1>); break;
            case 2: launch(ShadeIdsKernel<true, 2>); break;
            case 3: launch(ShadeIdsKernel<true, 3>); break;
            case 4: launch(ShadeIdsKernel<true, 4>); break;
            case 5: launch(ShadeIdsKernel<true, 5>); break;
            case 6: launch(ShadeIdsKernel<true, 6>); break;
            case 7: launch(ShadeIdsKernel<true, 7>); break;
            default: launch(ShadeIdsKernel<true, 8>); break;
        }
        static_assert(kMaxIdPlanes == 8, "one kernel per plane count");
    } else {
        hipLaunchKernelGGL((ShadeIdsKernel<false, 0>), grid, dim3(kShadeThreads), 0, stream, p, ids,
                           static_cast<unsigned>(band_rows), static_cast<unsigned>(frames),
                           static_cast<unsigned>(interleaved), offsets_stride / 2, skip,
                           static_cast<unsigned>(own_bands), size_t{0}, static_cast<unsigned>(first_rows));
    }
    return hipGetLastError();
}

}  // namespace srt
