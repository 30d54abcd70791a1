// Internal declarations shared by mgr_kernels.hip and mgr_capi.hip.
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "mgr.h"
#include "mgr_instrument.h"

namespace mgr {

constexpr int kBlock = 256;              // 4 waves of 64
constexpr int kWaves = kBlock / 64;
constexpr int kMaxTileRows = 65536;      // many-bin pack tiles (super-rounds of 4096 rows)
constexpr int kCoopMaxRounds = 64;       // cooperative pack tiles <= 4096 rows
constexpr int kLdsBudget = 78 * 1024;    // per pack workgroup: 2 workgroups per CU (160 KiB)
constexpr int kScanFlags = 4096;         // one-pass scan: chunks (= workgroups) at most
constexpr int kMaxSets = 32;           // multi-selection sets per pass (halo pieces <= 26)

// One-pass scan control words, right behind the kScanFlags chunk words and
// zeroed with them by every count producer.
struct ScanCtl {
    uint32_t ticket;   // chunk ids in dispatch order (atomic ticket)
    uint32_t err;      // nonzero: a look-back timed out; packs then write nothing
    uint64_t done;     // chunks that wrote their offsets (bits 0-31), failed ones (32-63)
};
constexpr int kScanCtlWords = sizeof(ScanCtl) / 8;

// Geometry of one plan, passed to kernels by value (kernarg segment).
struct Geom {
    int dim;
    int compute_f32;                     // numpy f32 % f32 semantics (S9 note)
    int nbins;
    int nbits;                           // ceil(log2(nbins)) for the ballot match
    int fast[MGR_MAX_DIM];               // L > 0 and 2L finite: [0,L) fast wrap is exact
    int fastf[MGR_MAX_DIM];
    double L[MGR_MAX_DIM];
    double twoL[MGR_MAX_DIM];
    float Lf[MGR_MAX_DIM];
    float twoLf[MGR_MAX_DIM];
    int pow2[MGR_MAX_DIM];               // L is a power of two: x / L == x * (1/L) exactly
    int pow2f[MGR_MAX_DIM];
    double invL[MGR_MAX_DIM];
    float invLf[MGR_MAX_DIM];
    double nd[MGR_MAX_DIM];              // (double)n[d], the int64 multiplier promoted
    int64_t n[MGR_MAX_DIM];
    int64_t off[MGR_MAX_DIM];            // row-major offsets, last axis fastest (S4)
    int fine;                            // fine-cell plan (mgr_plan_create_fine)
    int64_t fmod[MGR_MAX_DIM];           // fine cells per rank cell and dimension
    int fast32;                          // every n[d] < 2^30: in-box rows bin in 32-bit ints
    int write_back_all;                  // mgr_plan_set_write_back: every slab written back
    int box_dtype;                       // the caller's box_length dtype (mgr_dtype)
    // Per call, from the positions' dtype (mgr_capi.hip pos_modes; read by the
    // int32 / int64 / float16 positions' path, bin_coord_ext): numpy's result
    // type of `position[:, d] % box[d]` (MGR_F16/F32/F64/I32/I64) and of
    // `position[:, d] / box[d]` (MGR_F16/F32/F64).
    int wmode;
    int dmode;
    int64_t Li[MGR_MAX_DIM];             // integer box lengths (wmode I32 / I64)
};

// The fine cells a row falls in, inside its destination's cell (SURVEY f4,
// config 5): the reference's binning over the global grid topology * fine
// (n, nd), reduced to k % fmod per dimension, numbered row-major (off).
// Same box as the plan it travels with; taken from a mgr_plan_create_fine plan.
struct FineGeom {
    double nd[MGR_MAX_DIM];
    int64_t n[MGR_MAX_DIM];
    int64_t fmod[MGR_MAX_DIM];
    int64_t off[MGR_MAX_DIM];
    int nbins;
};

// The halo's face thresholds (redist.py:271-276) for every cell index:
// cell_length[d] (numpy's box/topology) and overload_lengths[d].
struct HaloGeom {
    double cl[MGR_MAX_DIM];
    double ol[MGR_MAX_DIM];
};

// Workspace carve for (n, nbins, tile_rows).
struct Workspace {
    int32_t* counts;     // [nbins][T] destination-major tile histogram
    int64_t* offsets;    // [nbins][T] exclusive scan of counts
    int64_t* bin_starts; // [nbins + 1]
    uint64_t* flags;     // [kScanFlags] one-pass scan chunk words + ScanCtl; zeroed
                         // by the count producers (bin_count, bin_ids, rank_ids, msel_count)
    const uint32_t* scan_err;  // &ScanCtl::err: packs return at once when set
    int64_t T;
    int64_t t0 = 0, tn = 0;    // the tiles [t0, t0 + tn) one pack launch covers (all: 0, T)
};
int64_t num_tiles(int64_t n, int tile_rows);
int64_t workspace_bytes(int64_t n, int nbins, int tile_rows);
Workspace carve(void* base, int64_t n, int nbins, int tile_rows);
int dest_bytes(int nbins);
int nbits_for(int nbins);

// Kernel ids for the profiler.
enum KernelId { K_BIN_COUNT, K_SCAN, K_PACK, K_CELL_IDS, K_BIN_IDS, K_CELLNUM_IDX, K_SYNTH,
                K_EXCHANGE, K_HALO, K_BIN_FINE, K_COUNT_IDS, K_PACK_FINE, K_PACK_NARROW,
                K_HALO_PACK, K_ONEPASS, K_NUM_KERNELS };
const char* kernel_name(int k);
void prof_begin(hipStream_t s, int k);
void prof_end(hipStream_t s, int k);

// Launchers (return hipError_t of the launch; validate arguments before calling).
hipError_t launch_bin_count(const Geom& g, void* pos, int pos_dtype, int64_t n, int64_t stride,
                            int periodic, void* dest, int tile_rows, const Workspace& ws,
                            hipStream_t s, const FineGeom* fg = nullptr,
                            uint16_t* side_out = nullptr, const HaloGeom* hg = nullptr);
hipError_t launch_msel_count(const uint16_t* flags, int64_t n, int nsets, const int* masks,
                             int tile_rows, const Workspace& ws, hipStream_t s);
hipError_t launch_msel_pack(int nfields, const void* const* srcs, const int64_t* row_bytes,
                            int64_t n, const uint16_t* flags, int nsets, const int* masks,
                            int tile_rows, const Workspace& ws, void* const* dsts, hipStream_t s,
                            int64_t cap_rows = -1);
hipError_t launch_count_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows,
                            const Workspace& ws, void* dest, uint32_t* bad, hipStream_t s);
hipError_t launch_rank_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows,
                           const Workspace& ws, uint16_t* slots, uint16_t* tile_starts,
                           uint32_t* bad, hipStream_t s);
hipError_t launch_pack_ranked(const void* src, int64_t row_bytes, int64_t n, const uint16_t* ids,
                              const uint16_t* ranks, const uint16_t* tile_starts, int nbins,
                              int tile_rows, const Workspace& ws, void* dst, hipStream_t s);
hipError_t launch_cell_ids(const Geom& g, void* pos, int pos_dtype, int64_t n, int64_t stride,
                           int periodic, int64_t* cell, int64_t* idx, hipStream_t s);
hipError_t launch_bin_ids(const void* ids, int ids_dtype, int64_t n, int nbins, void* dest,
                          int tile_rows, const Workspace& ws, hipStream_t s);
hipError_t launch_cellnum_from_idx(const Geom& g, const int64_t* idx, int64_t n, int periodic,
                                   int64_t* cell, hipStream_t s);
hipError_t launch_scan(int64_t n, int nbins, int tile_rows, const Workspace& ws,
                       int64_t* bin_counts, hipStream_t s);
hipError_t launch_pack(const void* src, int64_t row_bytes, int64_t n, const void* dest,
                       int nbins, int drop_bin, int tile_rows, const Workspace& ws, void* dst,
                       int redirect_bin, void* redirect_dst, hipStream_t s,
                       const uint16_t* ids_src = nullptr, uint16_t* ids_dst = nullptr,
                       uint16_t* ids_red = nullptr);
hipError_t launch_pack_fields(int nf, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                              const void* dest, int nbins, int drop_bin, int tile_rows,
                              const Workspace& ws, void* const* dsts, int redirect_bin,
                              void* const* reds, hipStream_t s, const uint16_t* ids_src,
                              uint16_t* ids_dst, uint16_t* ids_red);
hipError_t launch_synth_uniform(uint64_t seed, int64_t gid0, int64_t n, int dim,
                                const double* box, double* pos, void* rec32, hipStream_t s);
int pack_tile_rows(int64_t row_bytes, int nbins);
hipError_t launch_tile_offsets(const Workspace& ws, int nbins, const int64_t* tiles, int ntiles,
                               int64_t* out, hipStream_t s);
int ranked_tile_rows(int64_t row_bytes, int nbins);
// The plan's geometry class for bin_row_fast (kGeoAny / kGeoF32 / kGeoF64).
int geo_kind(const Geom& g, bool pos_f32);
// One-pass source partition (mgr_onepass.hip, mgr_partition_onepass).
int64_t onepass_workspace_bytes(int64_t n, int nbins);
hipError_t launch_onepass(const Geom& g, const FineGeom* fg, void* data, int64_t row_bytes,
                          int64_t pos_off, int pos_dtype, int64_t n, int periodic, void* out,
                          uint16_t* fine_out, int64_t cap, int64_t* bin_counts, void* workspace,
                          hipStream_t s);
hipError_t launch_halo_flags(const void* pos, int pos_dtype, int64_t n, int64_t stride, int dim,
                             const double* hi, const double* lo, uint16_t* flags, hipStream_t s);

// Test hooks (include/mgr_instrument.h, mgr_test_hook): switches that make a
// product-reachable fallback or shape run on inputs that would not take it,
// so the parity tests reach every path.  None changes results.  Launches read
// an immutable snapshot (hooks(), read ONCE per launcher: `const Hooks& h =
// hooks();`); mgr_test_hook publishes a new one as a whole, so a launch sees
// either the old or the new set, never a mix.  The
// shipped configuration is the default-constructed snapshot.
struct Hooks {
    int tile_rounds = 0;     // != 0: pack/bin tiles of 64 * tile_rounds rows
    int scan_chunk = 2048;   // one-pass scan: counts per chunk (8 per thread)
    int scan_max_chunks = 1024;  // one-pass scan: at most this many chunks (look-back depth)
    int scan_spins = 1 << 24;    // polls per look-back word before giving up (-1: at once)
    int pack_img_all = 0;    // image pack for every 4-byte-multiple row of 12..60 B (else 24..60)
    int rank_rows = 0;       // ranked fine sort tiles: 0 automatic, 2048, 4096
    int bin_unstaged = 0;    // bin kernel without LDS slab staging (the wide / unaligned fallback)
    int bin_generic = 0;     // bin kernel with run-time geometry also for simple plans
    int pack_generic = 0;    // wave-per-tile pack_kernel also for <= 64 bins (the > 64-B row path)
    // scan race test: the chunk that ends bin scan_delay_bin counts itself
    // done, then sleeps scan_delay_sleeps x s_sleep(127) before storing its
    // inclusive word;
    // scan_end_spins >= 0 bounds the last ticket's polls of the bin-end words
    // (0 = one look: the pre-round-4 reader, which then reports the race)
    int scan_delay_bin = -1;
    int scan_delay_sleeps = 0;
    int scan_end_spins = -1;
    int scan_poison_chunk = -1;   // >= 0: that scan chunk publishes poisoned (a failed scan)
    int fields_kernel = 0;        // multi-field packs: 0 product choice, 1 per-wave image,
                                  // 2 tile image, 3 cooperative (where they take the fields)
};
// The scan kernel's copy of the race-test hooks (kernel argument).
struct ScanTest {
    int delay_bin, delay_sleeps, end_spins, poison_chunk;
};
const Hooks& hooks();
int set_hook(const char* key, int64_t value);   // mgr_test_hook

// Shipped constants that were A/B knobs (DESIGN.md §3.3 records the A/Bs).
constexpr int kXcdPackChunk = 16;   // packs: tiles dealt to the XCDs in chunks of 16
constexpr int kImgRoundsPerWave = 2;  // image pack: 64-row rounds per wave

}  // namespace mgr
