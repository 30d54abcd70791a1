/*
 * mgr.h -- C ABI of libmgr.so, the MI355X (gfx950) particle -> Cartesian grid
 * of ranks redistribution library.
 *
 * Drop-in boundary for the hot path of dkorytov/mpi_grid_redistribute
 * (redist.py).  The reference is pure Python (mpi4py + numpy); its "FFI" for
 * this path is the set of numpy/mpi4py calls listed per entry point below.
 * The package's Python layer (mpi_grid_redistribute_amd/) keeps the reference
 * API (MPIGridRedistributor, redistribute_by_position, ...) and binds exactly
 * these symbols with ctypes.  No torch types cross this boundary: device
 * buffers are plain pointers (hipMalloc'd or torch-owned), sizes are int64,
 * streams are hipStream_t passed as void*.
 *
 * Conventions
 *   - every function returns int: MGR_OK (0) or a negative mgr_status; the
 *     message of the last failure on the calling thread is mgr_last_error();
 *   - everything that takes a stream is stream-ordered and asynchronous: no
 *     host synchronisation, no allocation (graph-capturable), except
 *     mgr_comm_* creation and the explicitly synchronous helpers noted below;
 *   - workspaces are caller-owned device memory sized by mgr_workspace_bytes;
 *   - a plan is immutable after creation and may be shared by streams; one
 *     workspace must not be used by two in-flight calls at once.
 */
#ifndef MGR_H_
#define MGR_H_

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MGR_MAX_DIM 8
#define MGR_MAX_BINS 4096
#define MGR_MAX_FIELDS 16
#define MGR_UNIQUE_ID_BYTES 128

typedef enum {
    MGR_OK = 0,
    MGR_EINVAL = -1,      /* bad argument (shape, dtype, size)             */
    MGR_EHIP = -2,        /* HIP runtime error                             */
    MGR_ERCCL = -3,       /* RCCL error                                    */
    MGR_EUNSUPPORTED = -4 /* valid request this build does not implement   */
} mgr_status;

/* Element types.  Positions and box_length: any of them (the reference
 * bins any numeric numpy column, redist.py:68-69; numpy's promotion of
 * position % box and position / box depends on both dtypes, S9/S11a).
 * Rank ids: MGR_F32, MGR_F64, MGR_I32, MGR_I64.                           */
typedef enum {
    MGR_F32 = 1,
    MGR_F64 = 2,
    MGR_I32 = 3,
    MGR_I64 = 4,
    MGR_F16 = 5,
    MGR_I8 = 6,
    MGR_I16 = 7,
    MGR_U8 = 8,
    MGR_U16 = 9,
    MGR_U32 = 10,
    MGR_U64 = 11,
    MGR_B8 = 12   /* numpy bool, one byte                                   */
} mgr_dtype;

typedef struct mgr_plan mgr_plan; /* grid geometry of one rank            */
typedef struct mgr_comm mgr_comm; /* native RCCL communicator (one/GPU)    */

const char* mgr_last_error(void);
const char* mgr_version(void);

/* ---------------------------------------------------------------- plan --
 * Replaces MPIGridRedistributor.__init__ (redist.py:16-61): row-major cell
 * offsets (redist.py:53-58), the box and topology.  box_dtype is the numpy
 * dtype of the caller's box_length (redist.py:46); with the positions' dtype
 * it decides, as numpy 2.2.6's promotion does, the type the wrap
 * (position % box) and the quotient (position / box) compute in: e.g.
 * float32 positions with a float32 / float16 / int8 / int16 box compute in
 * float32, with a float64 / int32 / int64 box in float64 (S9, S11a); integer
 * positions with an integer box wrap in integer arithmetic.  Integer box
 * lengths are passed as doubles and must be integral with |L| < 2^53.
 * nbins = number of destinations = comm size (redist.py:42, :196); cells >=
 * nbins are invalid (redist.py:43-44 asserts prod(topology) <= size).      */
int mgr_plan_create(int dim, const int64_t* grid_topology, const double* box_length,
                    int box_dtype, int nbins, mgr_plan** out);
/* Fine-cell plan (BASELINE config 5): the destination-side
 * stable sort of a rank's particles by the fine cell they fall in, for
 * particle-mesh deposition.  The fine cell of a position is the reference's
 * own binning (redist.py:63-90, S1-S3) over the global grid topology*fine,
 * reduced to the index inside the rank's cell, k_d % fine[d], and numbered
 * row-major over fine (last axis fastest).  nbins = prod(fine) <= 4096.
 * Use with mgr_bin_count (periodic = 0: the rows were already wrapped by the
 * redistribution; the indexes still wrap, :90), mgr_scan and mgr_pack.     */
int mgr_plan_create_fine(int dim, const int64_t* grid_topology, const int64_t* fine,
                         const double* box_length, int box_dtype, mgr_plan** out);
int mgr_plan_destroy(mgr_plan* plan);
/* Position write-back of the periodic wrap (redist.py:68, :328-329 mutate
 * `position` in place).  MGR_WRITE_BACK_CHANGED (default): a 64-row slab is
 * stored only if one of its coordinates changed under the wrap -- the bytes
 * in memory are the reference's either way.  MGR_WRITE_BACK_ALL: every slab
 * is stored, the cost fresh input pays (87.5 % of uniform in-box f64 rows
 * change under x + L - L); bench.py times this.  Per plan, not process-wide. */
enum { MGR_WRITE_BACK_CHANGED = 0, MGR_WRITE_BACK_ALL = 1 };
int mgr_plan_set_write_back(mgr_plan* plan, int mode);

/* Rows per tile used by the histogram / pack kernels for rows of at most
 * max_row_bytes bytes and nbins destinations (a multiple of 64 rows).      */
int mgr_tile_rows(int64_t max_row_bytes, int nbins);
/* Device workspace for n rows, nbins bins (incl. a drop bin if any).       */
int64_t mgr_workspace_bytes(int64_t n, int nbins, int tile_rows);
/* Byte width of the per-row destination array for nbins bins: 1, 2 or 4.  */
int mgr_dest_bytes(int nbins);

/* ------------------------------------------------- binning (hot path) --
 * redist.py:157 -> get_cell_number_from_position (:87-90)
 *   -> get_cell_indexes_from_position (:63-71): per coordinate
 *      t = ((x % L) + L) % L written back IN PLACE (:68, :328-329) when
 *      periodic, then trunc(t / L * n) (:69-70)
 *   -> get_cell_number_from_indexes(periodic=True) (:73-85, :90): floor-mod
 *      wrap of every index and the row-major dot.
 * Bit-exact with numpy 2.2.6 (NaN/out-of-range bins
 * like x86's INT64_MIN).  pos: n rows, row r coordinate d at
 * pos[r*row_stride + d] (elements), any mgr_dtype.  Positions other than
 * float32 / float64 follow numpy's promotion (see mgr_plan_create): the wrap
 * is computed in the promoted type and cast back on the in-place write-back
 * (float -> integer as numpy's x86 casts, -> float16 rounded to nearest even,
 * -> bool != 0), the bin reads the stored value back.
 *
 * mgr_bin_count : writes dest[r] (mgr_dest_bytes(nbins) wide) and the per
 *                 tile histogram into the workspace; feeds mgr_scan.
 * mgr_cell_ids  : writes int64 cell ids (and optionally (n,dim) int64 cell
 *                 indexes, get_cell_indexes_from_position's output) only.  */
int mgr_bin_count(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n, int64_t row_stride,
                  int periodic, void* dest, int tile_rows, void* workspace, void* stream);
int mgr_cell_ids(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n, int64_t row_stride,
                 int periodic, int64_t* cell_out, int64_t* idx_out, void* stream);
/* mgr_bin_count + the fine cell of every row inside its DESTINATION's cell
 * (fine_plan = mgr_plan_create_fine over the same topology and box): the
 * source side of config 5.  fine_ids[r] (uint16) is what mgr_bin_count with
 * fine_plan would give for the stored (wrapped) position -- same quotient
 * t/L, multiplied by topology*fine -- so the fine ids travel with the rows
 * (a 2-byte field through mgr_pack / the exchange) and the destination sorts
 * by them (mgr_count_ids + mgr_scan + mgr_pack) without binning again.      */
int mgr_bin_count_fine(const mgr_plan* plan, const mgr_plan* fine_plan, void* pos, int pos_dtype,
                       int64_t n, int64_t row_stride, int periodic, void* dest,
                       uint16_t* fine_ids, int tile_rows, void* workspace, void* stream);
/* Tile histogram of n uint16 bin ids (< nbins) for mgr_scan, and the ids as
 * the destination array of the following mgr_pack (dest: n entries of
 * mgr_dest_bytes(nbins) bytes).  An id >= nbins (e.g. of another fine grid)
 * is clamped to nbins - 1 -- no table is indexed out of range -- and sets
 * *bad_ids nonzero (bad_ids: a caller-zeroed device word, or NULL); the
 * caller then treats the counts as failed (-1), like a failed scan.        */
int mgr_count_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows, void* dest,
                  uint32_t* bad_ids, void* workspace, void* stream);

/* redist.py:169-198 (redistribute_by_cell_number): caller-supplied rank
 * ids (MGR_I32/MGR_I64/MGR_F32/MGR_F64); ids outside [0, nbins) -- and
 * non-integral float ids -- go to the drop bin nbins, never sent (S6).
 * The histogram has nbins+1 bins; pass nbins+1 to scan/pack.               */
int mgr_bin_ids(const mgr_plan* plan, const void* ids, int ids_dtype, int64_t n, void* dest,
                int tile_rows, void* workspace, void* stream);

/* get_cell_number_from_indexes (redist.py:73-85) on device: idx (n,dim)
 * int64.  periodic: floor-mod wrap (:83-84); else plain dot, and the
 * reference's range check (:78-81, '&' bug) selects nothing.             */
int mgr_cell_number_from_indexes(const mgr_plan* plan, const int64_t* idx, int64_t n,
                                 int periodic, int64_t* cell_out, void* stream);

/* ---------------------------------------------------------------- scan --
 * Device-wide exclusive scan of the destination-major tile histogram:
 * segment start of every (bin, tile), bin starts, and per-bin totals
 * (bin_counts, int64[nbins], device) = the element counts of the
 * reference's send_buff[i] (redist.py:195-198).  Consumes what a count
 * producer (mgr_bin_count / mgr_bin_ids / mgr_msel_count ...) left in the
 * workspace, including the zeroed one-pass scan words: one producer
 * launch precedes every scan on the same stream.
 * Failure: the scan never hangs the GPU.  If a look-back gives up (a chunk's
 * predecessor never published, knob "scan_spins"), every bin_counts entry and
 * bin_starts[nbins] become -1 and a flag in the workspace makes every later
 * mgr_pack on this workspace write nothing -- the caller sees the failure at
 * its count read instead of wrong offsets.                                */
int mgr_scan(int64_t n, int nbins, int tile_rows, void* workspace, int64_t* bin_counts,
             void* stream);

/* ---------------------------------------------------------------- pack --
 * Stable partition of n rows of row_bytes (opaque bytes, redist.py:197
 * data[rank_to_send==i] for every i, S6/S8) into dst, bin-major, original
 * order kept inside each bin.  Rows of bin drop_bin (or -1: none) are not
 * written.  Rows of redirect_bin (or -1) are written to redirect_dst
 * starting at its row 0 instead (the self segment goes straight into the
 * caller's output), and the bins after it move up to close its gap in dst
 * (dst then holds exactly the rows that travel, bin-major).  Call once per
 * field; all fields share dest/workspace.                                  */
int mgr_pack(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nbins,
             int drop_bin, int tile_rows, const void* workspace, void* dst, int redirect_bin,
             void* redirect_dst, void* stream);

/* mgr_pack plus a 2-byte side field moved alike in the same pass: ids_src[r]
 * (uint16, e.g. the fine cell of mgr_bin_count_fine) goes to ids_dst (or
 * ids_redirect_dst) at the row's slot.  Kernels that cannot carry it (many
 * bins, selections) run a second 2-byte pack.                             */
int mgr_pack_ids(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nbins,
                 int drop_bin, int tile_rows, const void* workspace, void* dst, int redirect_bin,
                 void* redirect_dst, const uint16_t* ids_src, uint16_t* ids_dst,
                 uint16_t* ids_redirect_dst, void* stream);

/* mgr_pack_ids (ids_src NULL: mgr_pack) of the tiles [tile_begin, tile_end)
 * only (0 <= begin <= end <= the tile count of n, tile_rows): the rows of
 * those tiles land at their final places, so a caller can pack the tiles in
 * chunks and start moving each chunk's completed segment prefixes (the
 * pipelined exchange, exchange.py) while the next chunk is packed.       */
int mgr_pack_tiles(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nbins,
                   int drop_bin, int tile_rows, const void* workspace, void* dst, int redirect_bin,
                   void* redirect_dst, const uint16_t* ids_src, uint16_t* ids_dst,
                   uint16_t* ids_redirect_dst, int64_t tile_begin, int64_t tile_end,
                   void* stream);
/* Multi-field (SoA) stable partition: the nfields payload arrays of the same
 * n rows -- e.g. positions, velocities, masses and ids as separate arrays --
 * partitioned by ONE destination array and ONE ranking, in one pass where
 * the fields allow (redist.py:195-198 applied to every field with the same
 * rank_to_send: the reference's own :160-164 pattern, which redistributes
 * `position` with the destinations computed for `data`).  Field f: srcs[f]
 * holds n rows of row_bytes[f] opaque bytes, its packed rows go to dsts[f]
 * (and its redirect_bin rows to redirect_dsts[f]) exactly as mgr_pack would
 * place them; ids_src (or NULL): an optional 2-byte side field moved alike
 * (mgr_pack_ids).  tile_end < 0: every tile; else only the tiles
 * [tile_begin, tile_end) (mgr_pack_tiles).  nfields <= MGR_MAX_FIELDS.
 * Fields of 4-byte-multiple rows on 16-byte aligned sources (4-byte aligned
 * outputs), <= 64 bins, move together in one launch of the multi-field
 * kernel (each destination byte read and ranked once); any other field is
 * packed on its own with the same destinations.                          */
int mgr_pack_fields(int nfields, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                    const void* dest, int nbins, int drop_bin, int tile_rows,
                    const void* workspace, void* const* dsts, int redirect_bin,
                    void* const* redirect_dsts, const uint16_t* ids_src, uint16_t* ids_dst,
                    uint16_t* ids_redirect_dst, int64_t tile_begin, int64_t tile_end,
                    void* stream);
/* After mgr_scan: out[i * nbins + b] (device int64) = the first row of bin b
 * at tile tiles[i] in the packed layout (tiles[i] = the tile count: the bin's
 * end), i.e. where a chunk of tiles starts inside every bin's segment.
 * tiles: host array, ntiles <= 4096.                                       */
int mgr_tile_offsets(const void* workspace, int64_t n, int nbins, int tile_rows,
                     const int64_t* tiles, int ntiles, int64_t* out, void* stream);

/* The destination-side fine sort in two light steps (config 5).
 * mgr_rank_ids : for n uint16 ids (< nbins), every row's rank among the rows
 *                of its id inside its tile (ranks, uint16 [n]), every tile's
 *                start of each id inside the tile (tile_starts, uint16
 *                [ceil(n / tile_rows)][nbins]), and the tile histogram in the
 *                workspace for mgr_scan (nbins <= 2048; tile_rows =
 *                mgr_ranked_tile_rows(...), i.e. 2048 or 4096; MGR_EINVAL
 *                otherwise).
 * mgr_pack_ranked: the stable partition of n rows of row_bytes by those ids
 *                (after mgr_scan), each row placed at tile_start + rank --
 *                no ranking in the pack.  Rows of 4-byte multiples <= 64 B,
 *                tile_rows = mgr_ranked_tile_rows(row_bytes, nbins) (the
 *                same value for the rank, the scan, the workspace and every
 *                field's pack); MGR_EUNSUPPORTED otherwise (use mgr_pack).   */
/* Tile rows of the ranked fine sort for rows of row_bytes (the widest field
 * packed) and nbins ids: 4096 when the tile's LDS image fits, else 2048; 0
 * when the ranked path does not take these rows.                          */
int mgr_ranked_tile_rows(int64_t row_bytes, int nbins);
int mgr_rank_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows, uint16_t* ranks,
                 uint16_t* tile_starts, uint32_t* bad_ids, void* workspace, void* stream);
int mgr_pack_ranked(const void* src, int64_t row_bytes, int64_t n, const uint16_t* ids,
                    const uint16_t* ranks, const uint16_t* tile_starts, int nbins, int tile_rows,
                    const void* workspace, void* dst, void* stream);

/* One call = bin_count + scan + pack of one field: the 1-GPU local stage
 * (bin + scan + stable pack, BASELINE config 2).  bin_offsets: int64
 * [nbins+1] device.                                                       */
int mgr_partition_by_position(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n,
                              int64_t row_stride, int periodic, const void* src,
                              int64_t row_bytes, void* dst, void* dest, int64_t* bin_counts,
                              int tile_rows, void* workspace, void* stream);
/* One-pass source partition of records that hold their own positions (the
 * 36-byte config-5 records with their f32 position view, S9; positions at
 * byte pos_offset of every row, float32 / float64, 3-D, <= 64 bins): bin,
 * rank and scatter in ONE read of the records -- the classic path (bin pass +
 * pack) reads the record lines twice.  The output is the reference's
 * send_buff list itself (redist.py:195-198): bin b's rows, in their original
 * order, from out + b * cap_rows * row_bytes (its fine cells -- fine_plan as
 * in mgr_bin_count_fine, else NULL -- from fine_out + b * cap_rows).
 * Positions are wrapped in place as mgr_bin_count does (S1).  bin_counts
 * (int64 [nbins], device) = the rows of every bin; rows at or beyond cap_rows
 * are NOT written, so a count above cap_rows means the caller redoes the
 * partition with the classic path (mgr_bin_count with periodic = 0 re-bins
 * the stored, wrapped positions identically, S2) -- or -1 everywhere when a
 * look-back gave up (nothing written).  Workspace: mgr_onepass_workspace_bytes
 * (zeroed by the call).  MGR_EUNSUPPORTED for shapes it does not take.      */
int64_t mgr_onepass_workspace_bytes(int64_t n, int nbins);
int mgr_partition_onepass(const mgr_plan* plan, const mgr_plan* fine_plan, void* data,
                          int64_t row_bytes, int64_t pos_offset, int pos_dtype, int64_t n,
                          int periodic, void* out, uint16_t* fine_out, int64_t cap_rows,
                          int64_t* bin_counts, void* workspace, void* stream);
/* bin starts (int64[nbins+1], device) left in the workspace by mgr_scan.   */
int mgr_bin_starts(int64_t n, int nbins, int tile_rows, const void* workspace,
                   const int64_t** out);

/* ---------------------------------------------------------- halo (f1) --
 * exchange_overload_by_position (redist.py:202-309), the overload/halo
 * exchange that redistribute_by_position runs when overload_lengths is set
 * (:161-166).  Per dimension d the reference selects the rows to send right
 * with position[:, d] > rank_cell_limits[d,1] - overload_lengths[d] (:271,
 * :274) and left with position[:, d] < rank_cell_limits[d,0] +
 * overload_lengths[d] (:272, :275), compared in float64 (numpy promotion of
 * the column, of any mgr_dtype, against a float64 scalar: integers above
 * 2^53 round to float64 as numpy converts them; NaN selects none).
 *
 * mgr_halo_flags  : one pass over n position rows; flags[r] (uint16) bit 2d =
 *                   coordinate d > hi[d], bit 2d+1 = coordinate d < lo[d].
 *                   hi/lo: host arrays of dim doubles.
 *                   (exchange_overload_by_position on caller rows).       */
int mgr_halo_flags(const void* pos, int pos_dtype, int64_t n, int64_t row_stride, int dim,
                   const double* hi, const double* lo, uint16_t* flags, void* stream);
/* The halo face flags computed by the binning kernel itself, against the
 * limits of the cell each row lands in: mgr_bin_count + flags[r] (uint16, the
 * layout of mgr_halo_flags) for cell_length[d] (numpy's box/topology,
 * redist.py:49-51) and overload_lengths[d].  The flags travel with the rows
 * (mgr_pack_ids) and equal mgr_halo_flags of the rank that receives them --
 * and of every neighbour they are forwarded to, whose cell differs from it
 * only in the dimension of the exchange -- so no rank re-reads positions.  */
int mgr_bin_count_halo(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n,
                       int64_t row_stride, int periodic, void* dest, uint16_t* flags,
                       const double* cell_length, const double* overload_lengths, int tile_rows,
                       void* workspace, void* stream);
/* Multi-selection: set k = the rows whose flags hold every bit of masks[k]
 * (nonzero uint16 masks, nsets <= 32; one bit: a face of the halo, several:
 * an edge or corner region; a row may be in several sets), all sets in one
 * pass.  mgr_msel_count
 * writes the per-(set, tile) counts for mgr_scan(n, nsets, ...) (bin_counts
 * = the set sizes); then mgr_msel_pack writes one field's selected rows (any
 * width): set k's rows, in row order, to dsts[k] (nsets device pointers; NULL
 * = set k not written).  The halo's sends of a dimension and direction
 * (redist.py:271-275) go straight to a neighbour's staging buffer or, for a
 * self-neighbour, into the halo store.                                    */
int mgr_msel_count(const uint16_t* flags, int64_t n, int nsets, const int* masks, int tile_rows,
                   void* workspace, void* stream);
int mgr_msel_pack(const void* src, int64_t row_bytes, int64_t n, const uint16_t* flags,
                  int nsets, const int* masks, int tile_rows, const void* workspace,
                  void* const* dsts, void* stream);
/* mgr_msel_pack of nfields (1..3) fields of the same rows in one pass (the
 * flags read and the sets listed once): srcs[f] rows of row_bytes[f]; set k
 * of field f goes to dsts[f * nsets + k]; field 0's NULLs decide which sets
 * are written.                                                            */
int mgr_msel_pack_fields(int nfields, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                         const uint16_t* flags, int nsets, const int* masks, int tile_rows,
                         const void* workspace, void* const* dsts, void* stream);
/* mgr_msel_pack_fields with the sets placed on the device: every set of
 * field f back to back from dsts[f] (nfields pointers), set k at the scan's
 * start of set k -- the caller needs no set sizes before the launch (the
 * one-rank halo launches it before its one host sync).  Rows at or beyond
 * cap_rows (>= 0) are not written; the caller compares the scanned total
 * with cap_rows afterwards.                                               */
int mgr_msel_pack_placed(int nfields, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                         const uint16_t* flags, int nsets, const int* masks, int tile_rows,
                         const void* workspace, void* const* dsts, int64_t cap_rows, void* stream);

/* ------------------------------------------------------------ exchange --
 * Replaces comm.alltoall(send_buff) + np.concatenate (redist.py:199):
 * RCCL over xGMI, one process per GPU.  The unique id is made on one rank
 * and broadcast by the caller (any channel).  mgr_comm_create is
 * collective and synchronous; it binds the current HIP device.            */
int mgr_comm_unique_id(void* out_id /* MGR_UNIQUE_ID_BYTES */);
int mgr_comm_create(const void* id, int nranks, int rank, mgr_comm** out);
int mgr_comm_destroy(mgr_comm* comm);
int mgr_comm_rank(const mgr_comm* comm);
int mgr_comm_size(const mgr_comm* comm);
/* Ranks in the communicator as RCCL itself counts them (ncclCommCount), < 0
 * on error: the scaling record checks it against the world size.          */
int mgr_comm_count(const mgr_comm* comm);
/* RCCL versions (major*10000 + minor*100 + patch): the headers libmgr.so was
 * built with, and the library loaded in this process (ncclGetVersion; in a
 * torch process, torch's bundled RCCL).  Host only.  mgr_comm_create refuses
 * a runtime of another major version or older than 2.18 (MGR_ERCCL, both
 * versions in the message): the RCCL calls used keep their ABI within that
 * range.                                                                   */
int mgr_rccl_version(int* compiled, int* runtime);

/* All-to-all of one int64 per peer (the count row): recv[s] = send_of_s[me]. */
int mgr_exchange_counts(mgr_comm* comm, const int64_t* send_counts, int64_t* recv_counts,
                        void* stream);

/* All-to-all of `width` int64 per peer in one RCCL group: row p of send
 * ([size][width], device) goes to peer p, row s of recv comes from peer s.
 * The pipelined exchange sends [total, chunk counts...] per peer, so the totals
 * and the per-chunk counts take one host sync (replaces redist.py:199's count
 * alltoall; the chunks have no reference counterpart). */
int mgr_exchange_count_rows(mgr_comm* comm, const int64_t* send, int64_t* recv, int width,
                            void* stream);

/* Grouped ncclSend/ncclRecv of nfields packed, bin-major fields.  Counts and
 * offsets are in ROWS and live on the host.  Rows from source s land at
 * recv[f] + recv_offsets[s]*row_bytes[f]: source order (S7).  skip_self:
 * the self segment is already in place (mgr_pack redirect), else it is
 * copied device-to-device on the stream.                                  */
int mgr_exchange_rows(mgr_comm* comm, int nfields, const void* const* send, void* const* recv,
                      const int64_t* row_bytes, const int64_t* send_counts,
                      const int64_t* send_offsets, const int64_t* recv_counts,
                      const int64_t* recv_offsets, int skip_self, void* stream);
/* The operation list mgr_exchange_rows issues for rank `rank` of `size`, in
 * issue order (host only, no GPU or communicator needed: the RCCL schedule
 * is testable on a CPU).  Peers in ring order from rank+1 (sends to
 * rank+j, receives from rank-j), fields in order within a peer; then the
 * self-segment copies when !skip_self.  Writes at most max_ops entries to
 * ops (may be NULL) and returns the total number of operations, < 0 on error.
 * Offsets and sizes are in bytes: src_offset into send[field] (SEND, COPY),
 * dst_offset into recv[field] (RECV, COPY).                                */
enum { MGR_XOP_SEND = 0, MGR_XOP_RECV = 1, MGR_XOP_COPY = 2 };
typedef struct {
    int32_t kind, peer, field, reserved;
    int64_t src_offset, dst_offset, bytes;
} mgr_xop;
int mgr_exchange_schedule(int rank, int size, int nfields, const int64_t* row_bytes,
                          const int64_t* send_counts, const int64_t* send_offsets,
                          const int64_t* recv_counts, const int64_t* recv_offsets, int skip_self,
                          mgr_xop* ops, int max_ops);
/* One group of point-to-point operations (kinds MGR_XOP_SEND / _RECV, byte
 * counts, device buffers), posted in order: RCCL matches a pair of ranks'
 * sends and receives in posting order, so the halo's two sequential steps
 * per dimension (redist.py:289-303) become one group when each rank posts
 * step 1 (send right, receive from left) before step 2.  Operations with
 * this rank as peer pair up in order as device copies.                     */
int mgr_group_p2p(mgr_comm* comm, int nops, const int* kinds, const int* peers,
                  void* const* bufs, const int64_t* bytes, void* stream);
/* Element-wise max all-reduce of count doubles (bench timing, barriers).   */
int mgr_comm_allreduce_max_f64(mgr_comm* comm, const double* in, double* out, int64_t count,
                               void* stream);

/* ------------------------------------------------------- synthetic data --
 * SURVEY §8d counter-based generator: u = (splitmix64(seed ^ (3*gid+d))
 * >> 11) * 2^-53, pos[i*dim+d] = u * box[d], gid = gid0 + i; optional
 * 32-byte records [x, y, z (f64), id (i64)] (dim must be 3).             */
int mgr_synth_uniform(uint64_t seed, int64_t gid0, int64_t n, int dim, const double* box,
                      double* pos, void* rec32, void* stream);

/* Measurement and test hooks (mgr_test_hook, mgr_profile_*) are not part of
 * the drop-in boundary: include/mgr_instrument.h.                          */

#ifdef __cplusplus
}
#endif
#endif /* MGR_H_ */
