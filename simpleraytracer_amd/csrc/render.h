// Host-side interface of the HIP render kernels (render.hip).
//
// Pipeline for one frame (or one row band of it), all on one HIP stream:
//   1. prepare: triangle list + frame -> per-triangle edge-function records (48 B each)
//   2. trace:   per pixel: primary ray from the sample offsets -> brute-force closest hit
//               over every triangle (LDS-tiled) -> shade -> RGBA float4 store
// The canonical arithmetic both kernels implement is specified in DESIGN.md "Canonical math"
// and restated independently by oracle/srt_oracle.c.
#pragma once

#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>

#include "scene.h"

namespace srt {

// Triangles per edge tile. The edge buffer is padded with disabled (all-NaN) records to a
// multiple of kPadTriangles (the largest cull step: 256 threads x 16 records) so no trace
// loop has a tail; the per-ray variants stop after the last tile holding a real record.
constexpr int kTileTriangles = 256;
constexpr int kPadTriangles = 4096;
// Floats per position of the scene's spatial-order record inputs (DeviceScene svertices): the 9
// vertex coordinates, the record id's bits, two zero words -- 48 B, three 16-B loads.
constexpr int kSpatialStride = 12;

// Edge records, tile-planar: tile t (256 records, 10 KiB) = four planes, each indexed by the
// record's position j in the tile, so a lane-per-record load is one coalesced 16-B or 4-B
// access per plane and an LDS copy of the tile is a straight 10 KiB memcpy.
//   plane 0: float4[256] (c0A, cxA, cyA, c0B)
//   plane 1: float4[256] (cxB, cyB, c0C, cxC)
//   plane 2: float [256] cyC
//   plane 3: float [256] vol
// E_k(fx, fy) = fma(fy, cy_k, fma(fx, cx_k, c0_k)) for the three edges k = A, B, C.
constexpr int kTileFloat4 = kTileTriangles * 5 / 2;  // 640 float4 = 10 KiB per tile

// Screen boxes (render.hip ScreenBox): one float4 (xlo, xhi, ylo, yhi) per record, in record
// order, right after the tiles. They bound only rays with |fx|, |fy| <= kScreenBoxRange.
constexpr float kScreenBoxRange = 4.0f;

// Quantized screen boxes (the cull kernel's streamed copy): one uint2 per record, in record
// order, after the float boxes: x = hi | (-lo) << 16, y likewise, as int16 fixed point
// q = v * kQuantScale, lo rounded down and hi up, clamped to [-32767, 32767].
constexpr float kQuantScale = 4096.0f;

// Cull records (render.hip CullRecord): 64 B per record, at the record's rank in the scene's
// spatial order, after the quantized boxes.
// Floats per record in the edge allocation: 10 (tiles) + 4 (screen box) + 2 (quantized box)
// + 16 (cull record). (Shading computes a hit triangle's normal from its vertices: no per-frame
// normal buffer -- round 2 scattered one, 16 B by triangle id, in every band's record pass.)
constexpr int kEdgeFloatsPerTriangle = 32;

inline std::uint64_t PaddedTriangleCount(std::uint64_t n) {
    const std::uint64_t p = (n + kPadTriangles - 1) / kPadTriangles * kPadTriangles;
    return p == 0 ? kPadTriangles : p;
}

// Trace kernel variants (DESIGN.md "Kernels"); selectable for A/B measurement.
enum TraceVariant : int {
    kTraceLds = 0,     // LDS-tiled triangle stream, every ray tests every record
    kTraceScalar = 1,  // wave-uniform scalar-cache triangle stream, no LDS, 1 wave per block
    kTraceCull = 2,    // hierarchical: block-box cull of every record, compacted survivors in LDS
    kTraceBvh = 3,     // screen-space 8-wide BVH over the records in spatial order, wave-packet traversal
};

struct BandArgs {
    const float* offsets;  // device, row_count x width x 2 (band-local rows)
    float* rgba;           // device, row_count x width x 4
    std::size_t width;
    std::size_t height;     // full frame height (fy denominator)
    std::size_t row_begin;  // first frame row of the band
    std::size_t row_count;
    int* ids = nullptr;     // device, row_count x width: non-null = store hit ids (-1 miss), not RGBA
    // The band's row pattern. 1: frame rows [row_begin, row_begin + row_count). P > 1: the band deals
    // the frame's tile rows (kCullTileRows each) round-robin over P bands: frame tile rows
    // row_begin / kCullTileRows + k P, k = 0, 1, ..., concatenated (row_begin a multiple of
    // kCullTileRows; only the band's last tile row may be partial, and then it is the frame's last).
    // RowPattern(P, g): g consecutive tile rows out of every P (the compositor's share, engine.h).
    std::size_t row_interleave = 1;
    // ids holds packed hit ids (PackedIds) with this many bit planes above the 16-bit low plane;
    // -1: int32 ids (-1 = miss). The multi-GPU exchange payload (cull variant).
    int id_planes = -1;
    // RGBA output only: rgba is the whole frame (height x width x 4) and band row y is stored at its
    // frame row (BandFrameRow) -- the compositor's own band traced straight into its frame.
    bool rgba_frame_rows = false;
};

// Packed hit ids (the multi-GPU exchange payload; cull variant): a pixel's code -- its triangle id, or
// all ones for a miss -- in 16 + k bits, k = the bits the triangle count needs beyond 16 (C3's 100 000
// triangles: 1, 2.125 B per pixel against int32's 4; under 65 535 triangles: 0; C5's 1M: 4). Row-major
// rows, each: the row's u16 low 16 bits (padded to 8 B), then per plane j one 64-bit word per 64
// columns (bit x % 64 of word x / 64 is bit 16 + j of pixel x's code). Rows come in tile rows of
// kCullTileRows, each followed by its tiles' sample offset: one float2 per 64-column tile, the
// offset every ray of the tile has (the tile is "regular"), or NaNs (0.4 % more bytes at 1080p), so
// the shading of a regular tile reads no per-pixel offsets. A band frame is its tile rows (padded to
// 256 B), so a band's actual rows and its buffer's rows index it alike. Written by the trace (one
// ballot per plane and row segment; the tile's offset by its first block), read by the deferred
// shading: no decode work.
constexpr int kMaxIdPlanes = 8;
int IdPlanes(std::uint64_t triangles);  // k; -1 when the ids need more than 16 + kMaxIdPlanes bits
struct PackedIds {
    int planes = 0;
    std::size_t rows = 0, width = 0;
    std::size_t words = 0;          // 64-bit words per row and plane
    std::size_t low_row_bytes = 0;  // a row's u16 values, padded to 8 B
    std::size_t row_bytes = 0;      // a row
    std::size_t tile_row_bytes = 0; // kCullTileRows rows, then words float2 tile offsets
    std::size_t bytes = 0;          // one band frame
};
PackedIds PackedIdLayout(int planes, std::size_t rows, std::size_t width);

// A band row pattern (BandArgs::row_interleave) taking `group` consecutive tile rows out of every
// `interleave`, group a power of two (the kernels split a band's tile row index with a shift and a
// mask, no division): interleave in the low 16 bits, log2(group) above (group 1: the plain interleave).
constexpr std::size_t RowPattern(std::size_t interleave, std::size_t group) {
    std::size_t log2 = 0;
    while ((std::size_t{2} << log2) <= group) {
        ++log2;
    }
    return interleave | log2 << 16;
}
// Frame row of band-local row `local` (BandArgs::row_interleave: an interleave or a RowPattern).
inline std::size_t BandFrameRow(std::size_t row_begin, std::size_t pattern, std::size_t local);
// Rows of the band of pattern `pattern` starting at frame row `row_begin` of a `height`-row frame.
std::size_t PatternBandRows(std::size_t height, std::size_t row_begin, std::size_t pattern);
// Whether a binned cull frame computes its tile info inside the bin launch (one launch fewer, the
// tile info and the bins concurrent): full frames (the band is the whole frame), unless env
// SRT_FUSED_INFO=0. Its bins then use the analytic tile bounds (valid for offsets in [0, 1]) and
// write every cull record; a frame with an offset outside [0, 1] streams every record in every
// tile (the work order sees the range tag), which is exact.
bool CullFusedInfo(std::size_t row_begin, std::size_t row_count, std::size_t height, std::size_t interleave);
// Whether a band fits a frame of `height` rows (row_count may be 0).
bool BandFits(std::size_t row_begin, std::size_t row_count, std::size_t interleave, std::size_t height);
// Rows of band `band` of `bands` interleaved bands of a `height`-row frame.
std::size_t InterleavedBandRows(std::size_t height, std::size_t bands, std::size_t band);

// Launch the prepare kernel: writes PaddedTriangleCount(n) / kTileTriangles tiles into `edges`,
// then the screen boxes, quantized boxes and cull records (d_rank: id -> spatial-order rank).
hipError_t LaunchPrepare(const float* d_vertices, const unsigned* d_rank, std::uint64_t n, const Frame& frame,
                         float* d_edges, hipStream_t stream, hipEvent_t ev_begin = nullptr,
                         hipEvent_t ev_end = nullptr);

// Cull tiles: 64 columns x 16 rows of rays, one trace block each (render.hip "Cull bins"; 32-row
// tiles of two 16-row trace blocks measured 3 % slower at C3: each block filtered the candidates of
// both halves).
constexpr int kCullTileCols = 64;
#ifndef SRT_TILE_ROWS
#define SRT_TILE_ROWS 16
#endif
constexpr int kCullTileRows = SRT_TILE_ROWS;

inline std::size_t BandFrameRow(std::size_t row_begin, std::size_t pattern, std::size_t local) {
    const std::size_t interleave = pattern & 0xFFFFu, log2 = pattern >> 16;
    const std::size_t lt = local / kCullTileRows;
    return row_begin + ((lt >> log2) * interleave + (lt & ((std::size_t{1} << log2) - 1))) * kCullTileRows +
           local % kCullTileRows;
}
constexpr int kMaxBatch = 8;          // frames of a batched cull launch with its parameters as kernel arguments
constexpr int kMaxBoundTiles = 2048;  // binning needs tiles_x + tiles_y <= this
constexpr int kMaxBinTiles = 8192;    // and tiles_x * tiles_y <= this (bin kernel LDS histogram)

// Work buffers of the cull variant's bins for one band shape (one allocation, carved by
// CullBinLayout; its first CullBinCounterBytes -- the counters, which reset themselves -- must be
// zero-filled when it is carved up for a shape; every other byte is written before it is read).
struct CullBins {
    const unsigned* order; // the scene's record ids in spatial order (DeviceScene; not in the buffer)
    const float* svertices;  // the scene's vertices in that order (DeviceScene; not in the buffer)
    // Per 256-position block of the spatial order: (lowest ylo, highest yhi) of its records' screen
    // boxes under the prepared frame (LaunchBlockExtents; DeviceScene). A band's record pass skips a
    // block whose extent meets none of its rows (a skip hint, exact: render.hip BandMayReach); null: none.
    const float2* block_ext = nullptr;
    void* tile_info;       // tiles x 32 B: ray box, uniform offset (TileInfoKernel)
    unsigned* counts;      // tiles + 1: list lengths, then the large-list length (this frame's buffer)
    unsigned* counts_next; // the slot's other count buffer (its next frame's): zeroed by this frame's trace
    unsigned* lists;       // tiles x capacity candidate ids (BinTrianglesKernel)
    unsigned* large_list;  // PaddedTriangleCount(n) ids binned to every tile
    void* work;            // trace work plan (WorkOrderKernel): descs descriptors, 32 B each
    unsigned* work_count;  // its length
    unsigned* arrive;      // per split slot: split chunks finished (self-resetting counters)
    void* split_keys;      // key slices of split parts: one per split slot (<= descs), 8 KiB each
    unsigned descs;        // trace grid = work descriptors per frame (<= CullDescriptors(tiles, 1))
    unsigned* range_tag;   // = gen when some sample offset of the frame lies outside [0, 1] (tile blocks)
    unsigned gen;          // the scene's frame number (never 0): tags are compared with it, not reset
    unsigned capacity;
    std::size_t tiles;
    bool plan = true;      // (re)build the slot's work plan with this frame (else the trace uses the last one)
    // Records recomputed by the trace (render.hip TraceRecords<true>): the bin launch writes a 16-B
    // screen box per position instead of the 64-B cull record, the trace rebuilds the record from the
    // scene's 48-B spatial inputs. Same frame bit for bit; trades bin-launch bytes for trace VALU, so
    // it pays where the bin launch is on the critical path (one frame queue, one-frame launches).
    // One value for every frame of a launch.
    bool recompute = false;
};
// Which records a DeviceScene's binned traces read (DeviceScene::SetRecordMode; env SRT_TRACE_RECORDS
// = stored | recompute | auto overrides): auto = recomputed for one-frame launches, stored otherwise.
enum RecordMode : int { kRecordsAuto = 0, kRecordsStored = 1, kRecordsRecompute = 2 };

// Tiles (64 x 32 rays) of a width x row_count band.
std::size_t CullTiles(std::size_t width, std::size_t row_count);

// Whether a band shape can be binned (its tile grid fits the bin kernel's LDS).
bool CullBinnable(std::size_t width, std::size_t row_count);

// Per-tile list capacity for n triangles (a list that overflows makes its tile stream every
// record; results are unaffected). Env SRT_CULL_BIN_CAP overrides it (tests).
unsigned CullBinCapacity(std::uint64_t n, std::size_t tiles);

// Trace grid of a band shape in a launch of `frames` frames: work descriptors per frame. A tile
// part's candidates may be cut into up to kMaxChunks chunks (blocks); WorkOrderKernel picks the
// chunk size so that a frame's descriptors fit. Room = max(parts x M, parts + E / frames): M =
// ceil(resident trace blocks / the launch's parts) (small bands: > 1), E = env SRT_CULL_SPLIT
// (default: the resident trace blocks) for cutting the heavy parts. Env SRT_CULL_CHUNKS = m
// forces parts x m (tests, measurement).
constexpr int kMaxChunks = 16;
unsigned CullDescriptors(std::size_t tiles, std::size_t frames);

// Bytes of the bin work buffer for n triangles and a band shape, and its carve-up.
std::size_t CullBinBytes(std::uint64_t n, std::size_t width, std::size_t row_count);
std::size_t CullBinCounterBytes(std::uint64_t n, std::size_t width, std::size_t row_count);  // the leading counters
// parity: which of the slot's two count buffers this frame bins into (alternate per frame of a slot).
CullBins CullBinLayout(void* base, std::uint64_t n, std::size_t width, std::size_t row_count, unsigned parity = 0);

// Optional stage timing events (null = not recorded). They are bound to the kernels' own
// dispatch packets (hipExtLaunchKernelGGL start / stop events), so timing adds no marker
// packets to the stream: `prep_*` = the prepare kernel (fused with the tile-info blocks in
// the binned cull variant: PrepareInfoKernel; TileInfoKernel alone when no prepare is
// pending), `bin_*` = BinTrianglesKernel (its last block also orders the tiles),
// `begin` / `end` = the trace kernel.
struct StageEvents {
    hipEvent_t prep_begin = nullptr;
    hipEvent_t prep_end = nullptr;
    hipEvent_t bin_begin = nullptr;
    hipEvent_t bin_end = nullptr;
    hipEvent_t begin = nullptr;
    hipEvent_t end = nullptr;
};

// Launch the trace kernel over one band (cull variant: bin + trace; bins == nullptr streams
// every record for every tile). prepare_rank != null: first (re)compute the edge records for
// `frame` (LaunchPrepare's work; fused with the tile-info blocks when binning).
hipError_t LaunchTrace(const float* d_edges, std::uint64_t n, const float* d_vertices, const float* d_shade,
                       const Frame& frame, const float background[3], const BandArgs& band, int variant,
                       const CullBins* bins, hipStream_t stream, const StageEvents* events = nullptr,
                       const unsigned* prepare_rank = nullptr, void* bvh = nullptr);

// Screen-space BVH (render.hip "BVH variant"): an implicit 8-wide tree over the cull records
// in spatial order. Level 0 node i = records [8i, 8i+8); level L node i = level L-1 nodes
// [8i, 8i+8); the top level has one node. Per node: screen box (float4) + depth lower bound.
constexpr int kBvhWidth = 8;
constexpr int kBvhMaxLevels = 16;
struct BvhLayout {
    unsigned levels = 0;                  // levels (the last one holds the root)
    unsigned count[kBvhMaxLevels] = {};   // nodes per level
    unsigned offset[kBvhMaxLevels] = {};  // first node of each level in the node arrays
    unsigned nodes = 0;                   // total
};
BvhLayout MakeBvhLayout(std::uint64_t n);
std::size_t BvhBytes(std::uint64_t n);  // node boxes (16 B) + depth bounds (4 B), 256-B aligned

// One frame of a batched cull launch: its edge-record slot, its bins (one band shape for the
// whole batch) and its band buffers.
struct CullFrame {
    const float* edges;
    const CullBins* bins;
    BandArgs band;
};
// Frames of one launch whose parameters travel in a device table instead of the kernel
// arguments (count > kMaxBatch): `device` and `host` (page-locked) of CullTableBytes(frames) bytes
// each, caller-owned. LaunchCullFrames fills `host` and uploads it to `device` on the stream; the
// caller must not rewrite `host` before that upload has executed (`uploaded`), and the stream order
// keeps the device copy alive for the launches that read it.
constexpr int kMaxTableFrames = 256;
struct CullTable {
    void* device;
    void* host;
    std::size_t frames;  // capacity
    // `host` as the device sees it (page-locked, mapped): the upload is then a small kernel reading it
    // over the bus instead of hipMemcpyAsync, which on ROCm 7.2 blocked the calling thread for 7 ms
    // at the first upload from some staging buffers (measured: tools/first_run_probe.py). Null: copy.
    const void* host_device = nullptr;
    // Recorded on the stream once the upload has read `host` (null: not recorded): the caller may
    // rewrite `host` after it, while the frames' launches still run.
    hipEvent_t uploaded = nullptr;
};
std::size_t CullTableBytes(std::size_t frames);

// The cull pipeline for `count` frames of one camera in four launches (tile info; record setup +
// bins; work lists; trace), block z of each working on frame z: the same per-frame work as
// `count` single-frame calls, with four launches per call. Up to kMaxBatch frames carry their
// parameters as kernel arguments; up to kMaxTableFrames through `table` (required then). The
// records are computed in the bin launch every call (bins->order: position -> id; d_rank unused).
// Events (optional): prep = tile info, bin = record setup + bins + work list, trace.
hipError_t LaunchCullFrames(const CullFrame* frames, std::size_t count, std::uint64_t n, const float* d_vertices,
                            const float* d_shade, const Frame& frame, const float background[3], const unsigned* d_rank,
                            hipStream_t stream, const StageEvents* events, const CullTable* table = nullptr);

// Deferred shading of a band from hit ids (band.ids) and sample offsets into band.rgba (normals
// from the vertices, d_edges unused): bit-identical to the fused trace.
// frames > 1 shades a batch whose ids are band-major, ids[band][frame][band_rows][width] (a
// gather of `frames` frames of band_rows-row bands; band_rows 0 = one band of row_count rows),
// into band.rgba[frame][row_count][width].
// interleaved > 0: the ids' bands are that many interleaved bands (BandArgs::row_interleave).
// offsets_stride: floats between consecutive frames' sample offsets (0: every frame of the batch
// shares band.offsets; a multiple of 2).
// The scene's shading table (once, at load): per triangle two float4, (the shading normal
// cross(v1 - v0, v2 - v0), its length) and (albedo, 0); d_table holds 8 floats per triangle. The
// d_shade arguments of the launches below take it.
// Screen-box y extent of every 256-position block of the spatial order under `frame` (records computed
// as the bin kernel computes them; n_pad / 256 float2 into d_ext): the band record pass's skip hint,
// keyed to (scene, camera, W x H) like the spatial order itself.
// Block extents LaunchBlockExtents writes for n triangles (one per bin block of the record pass:
// render.hip kBinThreads records each): the size of its d_ext.
std::size_t BlockExtentCount(std::uint64_t n);
hipError_t LaunchBlockExtents(const float* d_svertices, std::uint64_t n, const Frame& frame, float2* d_ext,
                              hipStream_t stream);
hipError_t LaunchShadeTable(const float* d_vertices, const float* d_albedo, std::uint64_t n, float* d_table,
                            hipStream_t stream);

hipError_t LaunchShade(const float* d_vertices, const float* d_shade, const float* d_edges, std::uint64_t n,
                       const Frame& frame, const float background[3], const BandArgs& band, hipStream_t stream,
                       std::size_t frames = 1, std::size_t band_rows = 0, std::size_t interleaved = 0,
                       std::size_t offsets_stride = 0, long skip_band = -1, std::size_t own_bands = 0,
                       std::size_t first_rows = 0);
// (skip_band >= 0: the rows of that band are left as they are; own_bands > 0: so are the rows of
// bands [0, own_bands), and the ids start at band own_bands -- the compositor's share, engine.h.
// first_rows > 0, contiguous bands only: band 0 has first_rows rows, the later ones band_rows each --
// BandSplit::first_rows.)

// Spatial order of the records (spatial.hip): ids sorted by the Morton code of their centroid's
// image-plane position under the scene camera, on the device (keys + rocPRIM radix sort), and
// its inverse; synchronous on `stream`. Optional events bracket the build (timing).
void BuildSpatialOrder(const float* d_vertices, std::uint64_t n, const Camera& camera, unsigned* d_order,
                       unsigned* d_rank, float* d_svertices, hipStream_t stream, hipEvent_t ev_begin = nullptr,
                       hipEvent_t ev_end = nullptr);

// Element-wise IEEE binary16 <-> binary32 conversion on the device (ML_FLOAT16 images):
// float -> half rounds to nearest even (overflow -> inf, NaN stays NaN); half -> float is exact.
// `half` buffers are uint16 bit patterns on the host side.
hipError_t LaunchFloatToHalf(const float* src, std::uint16_t* dst, std::size_t count, hipStream_t stream);
hipError_t LaunchHalfToFloat(const std::uint16_t* src, float* dst, std::size_t count, hipStream_t stream);

#ifdef SRT_DIAG
// Diagnostic build only: copy the cull kernel's per-block phase counters to host memory.
hipError_t DiagRead(void* host, std::size_t bytes);
#endif

}  // namespace srt
