// C ABI of libmgr.so (include/mgr.h): argument validation, plans,
// workspaces, the RCCL exchange, and the per-kernel HIP-event profiler.
#include <math.h>
#include <rccl/rccl.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <mutex>
#include <string>
#include <vector>

#include "mgr_internal.h"

#define MGR_VERSION_STRING "mgr 0.1.0 (gfx950)"

// ------------------------------------------------------------- errors
static thread_local std::string g_err;

static int fail(int code, const char* fmt, ...) {
    char buf[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return code;
}

#define HIP_OK(expr)                                                                  \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail(MGR_EHIP, "%s: %s (%s:%d)", #expr, hipGetErrorString(e_),     \
                        __FILE__, __LINE__);                                          \
    } while (0)

#define NCCL_OK(expr)                                                                 \
    do {                                                                              \
        ncclResult_t r_ = (expr);                                                     \
        if (r_ != ncclSuccess)                                                        \
            return fail(MGR_ERCCL, "%s: %s (%s:%d)", #expr, ncclGetErrorString(r_),   \
                        __FILE__, __LINE__);                                          \
    } while (0)

struct mgr_plan {
    mgr::Geom g;
};

struct mgr_comm {
    ncclComm_t nccl;
    int rank, size;
};

// ----------------------------------------------------------- profiler
namespace mgr {
namespace {
struct ProfRec {
    int kid;
    hipEvent_t a, b;
};
std::mutex g_prof_mu;
bool g_prof_on = false;
std::vector<ProfRec> g_pending;
std::vector<hipEvent_t> g_pool;
double g_ms[K_NUM_KERNELS];
int64_t g_cnt[K_NUM_KERNELS];
thread_local hipEvent_t t_open = nullptr;

hipEvent_t take_event() {
    if (!g_pool.empty()) {
        hipEvent_t e = g_pool.back();
        g_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreate(&e) != hipSuccess) return nullptr;
    return e;
}

void collect_locked() {
    for (auto& r : g_pending) {
        float ms = 0.f;
        if (hipEventSynchronize(r.b) == hipSuccess && hipEventElapsedTime(&ms, r.a, r.b) == hipSuccess) {
            g_ms[r.kid] += ms;
            g_cnt[r.kid] += 1;
        }
        g_pool.push_back(r.a);
        g_pool.push_back(r.b);
    }
    g_pending.clear();
}
}  // namespace

const char* kernel_name(int k) {
    static const char* names[K_NUM_KERNELS] = {"bin_count", "scan", "pack", "cell_ids",
                                               "bin_ids", "cellnum_idx", "synth",
                                               "exchange", "halo", "bin_fine", "count_ids",
                                               "pack_fine", "pack_narrow", "halo_pack",
                                               "onepass"};
    return (k >= 0 && k < K_NUM_KERNELS) ? names[k] : "?";
}

std::atomic<int64_t> g_prof_mask{-1};   // mgr_profile_select: bit k times kernel id k
static bool prof_selected(int k) { return g_prof_on && ((g_prof_mask.load(std::memory_order_relaxed) >> k) & 1); }

void prof_begin(hipStream_t s, int k) {
    if (!prof_selected(k)) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    t_open = take_event();
    if (t_open) (void)hipEventRecord(t_open, s);
}

void prof_end(hipStream_t s, int k) {
    if (!prof_selected(k) || !t_open) return;
    std::lock_guard<std::mutex> lk(g_prof_mu);
    hipEvent_t b = take_event();
    if (!b) return;
    (void)hipEventRecord(b, s);
    g_pending.push_back({k, t_open, b});
    t_open = nullptr;
    if (g_pending.size() > 4096) collect_locked();
}
}  // namespace mgr

// ============================================================== C ABI
extern "C" {

const char* mgr_last_error(void) { return g_err.c_str(); }
const char* mgr_version(void) { return MGR_VERSION_STRING; }

// numpy 2.2.6 dtype promotion (NEP 50, array with a numpy scalar of the box
// dtype: both strongly typed) over the element types of mgr_dtype.
struct Kind {
    char k;   // 'f', 'i', 'u'
    int bytes;
};
static bool dtype_kind(int t, Kind* out) {
    switch (t) {
        case MGR_F16: *out = {'f', 2}; return true;
        case MGR_F32: *out = {'f', 4}; return true;
        case MGR_F64: *out = {'f', 8}; return true;
        case MGR_I8: *out = {'i', 1}; return true;
        case MGR_I16: *out = {'i', 2}; return true;
        case MGR_I32: *out = {'i', 4}; return true;
        case MGR_I64: *out = {'i', 8}; return true;
        case MGR_U8: *out = {'u', 1}; return true;
        case MGR_U16: *out = {'u', 2}; return true;
        case MGR_U32: *out = {'u', 4}; return true;
        case MGR_U64: *out = {'u', 8}; return true;
        case MGR_B8: *out = {'b', 1}; return true;
        default: return false;
    }
}
static int dtype_of(Kind k) {
    if (k.k == 'f') return k.bytes == 2 ? MGR_F16 : k.bytes == 4 ? MGR_F32 : MGR_F64;
    if (k.k == 'i') return k.bytes == 1 ? MGR_I8 : k.bytes == 2 ? MGR_I16 : k.bytes == 4 ? MGR_I32 : MGR_I64;
    return k.bytes == 1 ? MGR_U8 : k.bytes == 2 ? MGR_U16 : k.bytes == 4 ? MGR_U32 : MGR_U64;
}
// numpy's result type of a op b for two of these element types.
static int promote(int a, int b) {
    Kind x, y;
    if (!dtype_kind(a, &x) || !dtype_kind(b, &y)) return 0;
    if (x.k == 'b' && y.k == 'b') return MGR_I8;   // bool % bool: numpy's int8 loop
    if (x.k == 'b') return b;                        // bool joins anything as that type
    if (y.k == 'b') return a;
    if (x.k == 'f' || y.k == 'f') {
        // an integer joins a float as the smallest float holding it exactly
        // (8-bit -> float16, 16-bit -> float32, wider -> float64)
        auto fw = [](Kind q) { return q.k == 'f' ? q.bytes : q.bytes == 1 ? 2 : q.bytes == 2 ? 4 : 8; };
        return dtype_of({'f', std::max(fw(x), fw(y))});
    }
    if (x.k == y.k) return dtype_of({x.k, std::max(x.bytes, y.bytes)});
    const Kind s = x.k == 'i' ? x : y, u = x.k == 'i' ? y : x;   // signed, unsigned
    if (s.bytes > u.bytes) return dtype_of(s);
    if (u.bytes < 8) return dtype_of({'i', 2 * u.bytes});
    return MGR_F64;   // int64 with uint64
}
static bool is_pos_dtype(int t) {
    Kind k;
    return dtype_kind(t, &k);   // every float, integer and bool dtype
}

// The per-call modes of a plan's geometry for positions of pos_dtype: the
// type of position % box (wmode) and of position / box (dmode: true
// division, float64 for two integers); compute_f32 = the float32 positions'
// path computes both in float32.
static void pos_modes(mgr::Geom& g, int pos_dtype) {
    g.wmode = promote(pos_dtype, g.box_dtype);
    Kind w;
    dtype_kind(g.wmode, &w);
    g.dmode = w.k == 'f' ? g.wmode : MGR_F64;
    g.compute_f32 = pos_dtype == MGR_F32 && g.wmode == MGR_F32;
}

int mgr_test_pos_modes(int pos_dtype, int box_dtype, int* wrap, int* quot) {
    Kind k;
    if (!dtype_kind(pos_dtype, &k) || !dtype_kind(box_dtype, &k) || !wrap || !quot)
        return fail(MGR_EINVAL, "pos_dtype %d, box_dtype %d", pos_dtype, box_dtype);
    mgr::Geom g{};
    g.box_dtype = box_dtype;
    pos_modes(g, pos_dtype);
    *wrap = g.wmode;
    *quot = g.dmode;
    return MGR_OK;
}

// Box geometry of a plan: L, 2L, fast-wrap and exact power-of-two division
// flags per dimension, integer lengths of an integer box, and the
// per-dimension cell counts n[d].
static int fill_box(mgr::Geom& g, int dim, const int64_t* n, const double* box, int box_dtype) {
    Kind bk;
    if (!dtype_kind(box_dtype, &bk)) return fail(MGR_EINVAL, "box_dtype %d", box_dtype);
    g.dim = dim;
    g.box_dtype = box_dtype;
    pos_modes(g, MGR_F64);   // per call: pos_modes for the positions' dtype
    for (int d = 0; d < dim; ++d) {
        if (n[d] < 1) return fail(MGR_EINVAL, "grid_topology[%d] = %lld < 1", d, (long long)n[d]);
        const double L = box[d];
        if (bk.k != 'f') {
            if (!(L == floor(L) && fabs(L) < 9007199254740992.0))
                return fail(MGR_EINVAL, "integer box_length[%d] = %g: not an integer below 2^53", d, L);
            g.Li[d] = (int64_t)L;
        }
        g.L[d] = L;
        g.twoL[d] = L + L;
        g.fast[d] = (L > 0.0) && isfinite(L + L);
        const float Lf = (float)L;
        g.Lf[d] = Lf;
        g.twoLf[d] = Lf + Lf;
        g.fastf[d] = (Lf > 0.0f) && isfinite(Lf + Lf);
        g.n[d] = n[d];
        g.nd[d] = (double)n[d];
        int e;
        g.pow2[d] = L > 0.0 && isfinite(L) && frexp(L, &e) == 0.5 && isnormal(1.0 / L);
        g.invL[d] = g.pow2[d] ? 1.0 / L : 0.0;
        g.pow2f[d] = Lf > 0.0f && isfinite(Lf) && frexpf(Lf, &e) == 0.5f && isnormal(1.0f / Lf);
        g.invLf[d] = g.pow2f[d] ? 1.0f / Lf : 0.0f;
    }
    g.fast32 = 1;
    for (int d = 0; d < dim; ++d)
        if (n[d] >= ((int64_t)1 << 30)) g.fast32 = 0;
    return MGR_OK;
}

int mgr_plan_create(int dim, const int64_t* topo, const double* box, int box_dtype, int nbins,
                    mgr_plan** out) {
    if (!out || !topo || !box) return fail(MGR_EINVAL, "null argument");
    if (dim < 1 || dim > MGR_MAX_DIM) return fail(MGR_EINVAL, "dim %d not in [1, %d]", dim, MGR_MAX_DIM);
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d not in [1, %d]", nbins, MGR_MAX_BINS);
    mgr::Geom g;
    memset(&g, 0, sizeof g);
    int rc = fill_box(g, dim, topo, box, box_dtype);
    if (rc) return rc;
    g.nbins = nbins;
    g.nbits = mgr::nbits_for(nbins);
    int64_t prod = 1;
    for (int d = dim - 1; d >= 0; --d) {
        g.off[d] = prod;
        prod *= topo[d];
        if (prod > nbins)
            return fail(MGR_EINVAL, "topology needs %lld ranks, have %d (redist.py:43-44)",
                        (long long)prod, nbins);
    }
    mgr_plan* p = new mgr_plan;
    p->g = g;
    *out = p;
    return MGR_OK;
}

int mgr_plan_create_fine(int dim, const int64_t* topo, const int64_t* fine, const double* box,
                         int box_dtype, mgr_plan** out) {
    if (!out || !topo || !fine || !box) return fail(MGR_EINVAL, "null argument");
    if (dim < 1 || dim > MGR_MAX_DIM) return fail(MGR_EINVAL, "dim %d not in [1, %d]", dim, MGR_MAX_DIM);
    mgr::Geom g;
    memset(&g, 0, sizeof g);
    int64_t global[MGR_MAX_DIM];
    int64_t nb = 1;
    for (int d = 0; d < dim; ++d) {
        if (topo[d] < 1 || fine[d] < 1)
            return fail(MGR_EINVAL, "topology and fine cells must be >= 1 (dim %d)", d);
        if (topo[d] > ((int64_t)1 << 31) || fine[d] > MGR_MAX_BINS)
            return fail(MGR_EINVAL, "topology/fine cells too large (dim %d)", d);
        global[d] = topo[d] * fine[d];
        nb *= fine[d];
        if (nb > MGR_MAX_BINS) return fail(MGR_EINVAL, "more than %d fine cells", MGR_MAX_BINS);
    }
    // the reference's binning over the global fine grid topology * fine ...
    int rc = fill_box(g, dim, global, box, box_dtype);
    if (rc) return rc;
    // ... then the index inside the rank's cell, row-major over fine
    g.fine = 1;
    int64_t off = 1;
    for (int d = dim - 1; d >= 0; --d) {
        g.fmod[d] = fine[d];
        g.off[d] = off;
        off *= fine[d];
    }
    g.nbins = (int)nb;
    g.nbits = mgr::nbits_for((int)nb);
    mgr_plan* p = new mgr_plan;
    p->g = g;
    *out = p;
    return MGR_OK;
}

int mgr_plan_destroy(mgr_plan* plan) {
    delete plan;
    return MGR_OK;
}

int mgr_plan_set_write_back(mgr_plan* plan, int mode) {
    if (!plan) return fail(MGR_EINVAL, "null plan");
    if (mode != MGR_WRITE_BACK_CHANGED && mode != MGR_WRITE_BACK_ALL)
        return fail(MGR_EINVAL, "write-back mode %d", mode);
    plan->g.write_back_all = mode == MGR_WRITE_BACK_ALL;
    return MGR_OK;
}

int mgr_tile_rows(int64_t max_row_bytes, int nbins) {
    if (max_row_bytes < 1) max_row_bytes = 1;
    return mgr::pack_tile_rows(max_row_bytes, nbins);
}

int mgr_ranked_tile_rows(int64_t row_bytes, int nbins) {
    return mgr::ranked_tile_rows(row_bytes, nbins);
}

int64_t mgr_workspace_bytes(int64_t n, int nbins, int tile_rows) {
    if (n < 0 || nbins < 1 || tile_rows < 64) return -1;
    return mgr::workspace_bytes(n, nbins, tile_rows);
}

int mgr_dest_bytes(int nbins) { return mgr::dest_bytes(nbins); }

static int check_tile(int tile_rows) {
    if (tile_rows < 64 || tile_rows > mgr::kMaxTileRows || tile_rows % 64)
        return fail(MGR_EINVAL, "tile_rows %d must be a multiple of 64 in [64, %d]", tile_rows,
                    mgr::kMaxTileRows);
    return MGR_OK;
}

static int check_pos(const mgr_plan* plan, const void* pos, int dtype, int64_t n, int64_t stride) {
    if (!plan) return fail(MGR_EINVAL, "null plan");
    if (!is_pos_dtype(dtype))
        return fail(MGR_EINVAL, "positions must be a float, integer or bool dtype (dtype %d)", dtype);
    if (n < 0) return fail(MGR_EINVAL, "n < 0");
    if (n > 0 && !pos) return fail(MGR_EINVAL, "null positions");
    if (stride < plan->g.dim) return fail(MGR_EINVAL, "row_stride %lld < dim %d", (long long)stride, plan->g.dim);
    return MGR_OK;
}

int mgr_bin_count(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n, int64_t row_stride,
                  int periodic, void* dest, int tile_rows, void* workspace, void* stream) {
    int rc = check_pos(plan, pos, pos_dtype, n, row_stride);
    if (rc) return rc;
    if ((rc = check_tile(tile_rows))) return rc;
    if (n > 0 && (!dest || !workspace)) return fail(MGR_EINVAL, "null dest/workspace");
    mgr::Geom g = plan->g;
    pos_modes(g, pos_dtype);
    const mgr::Workspace ws = mgr::carve(workspace, n, g.nbins, tile_rows);
    HIP_OK(mgr::launch_bin_count(g, pos, pos_dtype, n, row_stride, periodic, dest,
                                 tile_rows, ws, (hipStream_t)stream));
    return MGR_OK;
}

// The fine geometry of fine_plan over plan (same box and dimension,
// topology * fine), for the bin kernels' fine side output.
static int fine_geom(const mgr_plan* plan, const mgr_plan* fine_plan, mgr::Geom& g,
                     mgr::FineGeom& fg) {
    if (!fine_plan || !fine_plan->g.fine) return fail(MGR_EINVAL, "fine_plan is not a fine-cell plan");
    if (fine_plan->g.dim != plan->g.dim) return fail(MGR_EINVAL, "plans of different dimensions");
    for (int d = 0; d < plan->g.dim; ++d)
        if (memcmp(&fine_plan->g.L[d], &plan->g.L[d], sizeof(double)) ||
            fine_plan->g.n[d] != plan->g.n[d] * fine_plan->g.fmod[d] ||
            fine_plan->g.box_dtype != plan->g.box_dtype)
            return fail(MGR_EINVAL, "fine_plan is not over this plan's box and topology (dim %d)", d);
    memset(&fg, 0, sizeof fg);
    for (int d = 0; d < g.dim; ++d) {
        fg.nd[d] = fine_plan->g.nd[d];
        fg.n[d] = fine_plan->g.n[d];
        fg.fmod[d] = fine_plan->g.fmod[d];
        fg.off[d] = fine_plan->g.off[d];
    }
    fg.nbins = fine_plan->g.nbins;
    if (!fine_plan->g.fast32) g.fast32 = 0;   // the fine indexes must fit 32 bits too
    return MGR_OK;
}

int mgr_bin_count_fine(const mgr_plan* plan, const mgr_plan* fine_plan, void* pos, int pos_dtype,
                       int64_t n, int64_t row_stride, int periodic, void* dest,
                       uint16_t* fine_ids, int tile_rows, void* workspace, void* stream) {
    int rc = check_pos(plan, pos, pos_dtype, n, row_stride);
    if (rc) return rc;
    if ((rc = check_tile(tile_rows))) return rc;
    mgr::Geom g = plan->g;
    pos_modes(g, pos_dtype);
    mgr::FineGeom fg;
    if ((rc = fine_geom(plan, fine_plan, g, fg))) return rc;
    if (n > 0 && (!dest || !workspace || !fine_ids)) return fail(MGR_EINVAL, "null dest/fine_ids/workspace");
    const mgr::Workspace ws = mgr::carve(workspace, n, g.nbins, tile_rows);
    HIP_OK(mgr::launch_bin_count(g, pos, pos_dtype, n, row_stride, periodic, dest,
                                 tile_rows, ws, (hipStream_t)stream, &fg, fine_ids));
    return MGR_OK;
}

int mgr_bin_count_halo(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n,
                       int64_t row_stride, int periodic, void* dest, uint16_t* flags,
                       const double* cell_length, const double* overload_lengths, int tile_rows,
                       void* workspace, void* stream) {
    int rc = check_pos(plan, pos, pos_dtype, n, row_stride);
    if (rc) return rc;
    if ((rc = check_tile(tile_rows))) return rc;
    if (plan->g.fine) return fail(MGR_EINVAL, "a fine-cell plan has no halo");
    if (!cell_length || !overload_lengths) return fail(MGR_EINVAL, "null cell/overload lengths");
    if (n > 0 && (!dest || !workspace || !flags)) return fail(MGR_EINVAL, "null dest/flags/workspace");
    mgr::Geom g = plan->g;
    pos_modes(g, pos_dtype);
    mgr::HaloGeom hg;
    memset(&hg, 0, sizeof hg);
    for (int d = 0; d < g.dim; ++d) {
        hg.cl[d] = cell_length[d];
        hg.ol[d] = overload_lengths[d];
    }
    const mgr::Workspace ws = mgr::carve(workspace, n, g.nbins, tile_rows);
    HIP_OK(mgr::launch_bin_count(g, pos, pos_dtype, n, row_stride, periodic, dest,
                                 tile_rows, ws, (hipStream_t)stream, nullptr, flags, &hg));
    return MGR_OK;
}

static int check_sets(int nsets, const int* masks) {
    if (nsets < 1 || nsets > mgr::kMaxSets || !masks)
        return fail(MGR_EINVAL, "nsets %d (1..%d)", nsets, mgr::kMaxSets);
    for (int k = 0; k < nsets; ++k)
        if (masks[k] < 1 || masks[k] > 0xFFFF) return fail(MGR_EINVAL, "set %d: flag mask %d", k, masks[k]);
    return MGR_OK;
}

int mgr_msel_count(const uint16_t* flags, int64_t n, int nsets, const int* masks, int tile_rows,
                   void* workspace, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc || (rc = check_sets(nsets, masks))) return rc;
    if (n < 0) return fail(MGR_EINVAL, "n < 0");
    if (n > 0 && (!flags || !workspace)) return fail(MGR_EINVAL, "null argument");
    const mgr::Workspace ws = mgr::carve(workspace, n, nsets, tile_rows);
    HIP_OK(mgr::launch_msel_count(flags, n, nsets, masks, tile_rows, ws, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_msel_pack(const void* src, int64_t row_bytes, int64_t n, const uint16_t* flags,
                  int nsets, const int* masks, int tile_rows, const void* workspace,
                  void* const* dsts, void* stream) {
    return mgr_msel_pack_fields(1, &src, &row_bytes, n, flags, nsets, masks, tile_rows, workspace,
                                dsts, stream);
}

int mgr_msel_pack_fields(int nfields, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                         const uint16_t* flags, int nsets, const int* masks, int tile_rows,
                         const void* workspace, void* const* dsts, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc || (rc = check_sets(nsets, masks))) return rc;
    if (nfields < 1 || nfields > 3 || !srcs || !row_bytes)
        return fail(MGR_EINVAL, "nfields %d (1..3)", nfields);
    for (int f = 0; f < nfields; ++f)
        if (row_bytes[f] < 1) return fail(MGR_EINVAL, "row_bytes %lld", (long long)row_bytes[f]);
    if (n > 0 && (!flags || !workspace || !dsts)) return fail(MGR_EINVAL, "null argument");
    for (int f = 0; n > 0 && f < nfields; ++f)
        if (!srcs[f]) return fail(MGR_EINVAL, "null argument");
    if (n <= 0) return MGR_OK;
    const mgr::Workspace ws = mgr::carve((void*)workspace, n, nsets, tile_rows);
    HIP_OK(mgr::launch_msel_pack(nfields, srcs, row_bytes, n, flags, nsets, masks, tile_rows, ws,
                                 dsts, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_msel_pack_placed(int nfields, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                         const uint16_t* flags, int nsets, const int* masks, int tile_rows,
                         const void* workspace, void* const* dsts, int64_t cap_rows, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc || (rc = check_sets(nsets, masks))) return rc;
    if (nfields < 1 || nfields > 3 || !srcs || !row_bytes)
        return fail(MGR_EINVAL, "nfields %d (1..3)", nfields);
    if (cap_rows < 0) return fail(MGR_EINVAL, "cap_rows %lld", (long long)cap_rows);
    for (int f = 0; f < nfields; ++f)
        if (row_bytes[f] < 1) return fail(MGR_EINVAL, "row_bytes %lld", (long long)row_bytes[f]);
    if (n > 0 && (!flags || !workspace || !dsts)) return fail(MGR_EINVAL, "null argument");
    for (int f = 0; n > 0 && f < nfields; ++f)
        if (!srcs[f] || (cap_rows > 0 && !dsts[f])) return fail(MGR_EINVAL, "null argument");
    if (n <= 0 || cap_rows == 0) return MGR_OK;
    const mgr::Workspace ws = mgr::carve((void*)workspace, n, nsets, tile_rows);
    HIP_OK(mgr::launch_msel_pack(nfields, srcs, row_bytes, n, flags, nsets, masks, tile_rows, ws,
                                 dsts, (hipStream_t)stream, cap_rows));
    return MGR_OK;
}

int mgr_count_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows, void* dest,
                  uint32_t* bad_ids, void* workspace, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (n < 0) return fail(MGR_EINVAL, "n < 0");
    if (n > 0 && (!ids || !workspace || !dest)) return fail(MGR_EINVAL, "null argument");
    const mgr::Workspace ws = mgr::carve(workspace, n, nbins, tile_rows);
    HIP_OK(mgr::launch_count_ids(ids, n, nbins, tile_rows, ws, dest, bad_ids, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_rank_ids(const uint16_t* ids, int64_t n, int nbins, int tile_rows, uint16_t* ranks,
                 uint16_t* tile_starts, uint32_t* bad_ids, void* workspace, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    // the ranked tiles only (mgr_ranked_tile_rows: 2048 or 4096 rows, <= 2048
    // ids: the per-wave LDS peer words); anything else is refused here, not
    // by the launch
    if (nbins < 1 || nbins > 2048) return fail(MGR_EINVAL, "nbins %d not in [1, 2048]", nbins);
    if (tile_rows != 2048 && tile_rows != 4096)
        return fail(MGR_EINVAL, "tile_rows %d: 2048 or 4096 (mgr_ranked_tile_rows)", tile_rows);
    if (n < 0) return fail(MGR_EINVAL, "n < 0");
    if (n > 0 && (!ids || !ranks || !tile_starts || !workspace)) return fail(MGR_EINVAL, "null argument");
    const mgr::Workspace ws = mgr::carve(workspace, n, nbins, tile_rows);
    HIP_OK(mgr::launch_rank_ids(ids, n, nbins, tile_rows, ws, ranks, tile_starts, bad_ids,
                                (hipStream_t)stream));
    return MGR_OK;
}

int mgr_pack_ranked(const void* src, int64_t row_bytes, int64_t n, const uint16_t* ids,
                    const uint16_t* ranks, const uint16_t* tile_starts, int nbins, int tile_rows,
                    const void* workspace, void* dst, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (row_bytes < 1) return fail(MGR_EINVAL, "row_bytes %lld", (long long)row_bytes);
    if (n > 0 && (!src || !ids || !ranks || !tile_starts || !workspace || !dst))
        return fail(MGR_EINVAL, "null argument");
    const mgr::Workspace ws = mgr::carve((void*)workspace, n, nbins, tile_rows);
    const hipError_t e = mgr::launch_pack_ranked(src, row_bytes, n, ids, ranks, tile_starts, nbins,
                                                 tile_rows, ws, dst, (hipStream_t)stream);
    if (e == hipErrorNotSupported)
        return fail(MGR_EUNSUPPORTED, "ranked pack: rows of %lld bytes, tile_rows %d (needs 4-byte "
                    "multiples <= 64, tile_rows = mgr_tile_rows, 4-byte aligned buffers)",
                    (long long)row_bytes, tile_rows);
    HIP_OK(e);
    return MGR_OK;
}

int mgr_cell_ids(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n, int64_t row_stride,
                 int periodic, int64_t* cell_out, int64_t* idx_out, void* stream) {
    int rc = check_pos(plan, pos, pos_dtype, n, row_stride);
    if (rc) return rc;
    mgr::Geom g = plan->g;
    pos_modes(g, pos_dtype);
    HIP_OK(mgr::launch_cell_ids(g, pos, pos_dtype, n, row_stride, periodic, cell_out,
                                idx_out, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_bin_ids(const mgr_plan* plan, const void* ids, int ids_dtype, int64_t n, void* dest,
                int tile_rows, void* workspace, void* stream) {
    if (!plan) return fail(MGR_EINVAL, "null plan");
    if (ids_dtype < MGR_F32 || ids_dtype > MGR_I64) return fail(MGR_EINVAL, "ids dtype %d", ids_dtype);
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (n > 0 && (!ids || !dest || !workspace)) return fail(MGR_EINVAL, "null argument");
    if (plan->g.nbins + 1 > MGR_MAX_BINS) return fail(MGR_EINVAL, "too many bins");
    const mgr::Workspace ws = mgr::carve(workspace, n, plan->g.nbins + 1, tile_rows);
    HIP_OK(mgr::launch_bin_ids(ids, ids_dtype, n, plan->g.nbins, dest, tile_rows, ws,
                               (hipStream_t)stream));
    return MGR_OK;
}

int mgr_cell_number_from_indexes(const mgr_plan* plan, const int64_t* idx, int64_t n,
                                 int periodic, int64_t* cell_out, void* stream) {
    if (!plan) return fail(MGR_EINVAL, "null plan");
    if (n > 0 && (!idx || !cell_out)) return fail(MGR_EINVAL, "null argument");
    HIP_OK(mgr::launch_cellnum_from_idx(plan->g, idx, n, periodic, cell_out, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_scan(int64_t n, int nbins, int tile_rows, void* workspace, int64_t* bin_counts,
             void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (!workspace) return fail(MGR_EINVAL, "null workspace");
    const mgr::Workspace ws = mgr::carve(workspace, n, nbins, tile_rows);
    HIP_OK(mgr::launch_scan(n, nbins, tile_rows, ws, bin_counts, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_bin_starts(int64_t n, int nbins, int tile_rows, const void* workspace,
                   const int64_t** out) {
    if (!workspace || !out) return fail(MGR_EINVAL, "null argument");
    *out = mgr::carve((void*)workspace, n, nbins, tile_rows).bin_starts;
    return MGR_OK;
}

int mgr_pack(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nbins,
             int drop_bin, int tile_rows, const void* workspace, void* dst, int redirect_bin,
             void* redirect_dst, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (row_bytes < 1) return fail(MGR_EINVAL, "row_bytes %lld", (long long)row_bytes);
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (n > 0 && (!src || !dest || !workspace)) return fail(MGR_EINVAL, "null argument");
    if (n > 0 && redirect_bin >= 0 && !redirect_dst) return fail(MGR_EINVAL, "redirect without buffer");
    if (redirect_bin >= nbins) return fail(MGR_EINVAL, "redirect_bin out of range");
    const mgr::Workspace ws = mgr::carve((void*)workspace, n, nbins, tile_rows);
    HIP_OK(mgr::launch_pack(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst,
                            redirect_bin, redirect_dst, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_pack_ids(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nbins,
                 int drop_bin, int tile_rows, const void* workspace, void* dst, int redirect_bin,
                 void* redirect_dst, const uint16_t* ids_src, uint16_t* ids_dst,
                 uint16_t* ids_redirect_dst, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (row_bytes < 1) return fail(MGR_EINVAL, "row_bytes %lld", (long long)row_bytes);
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (n > 0 && (!src || !dest || !workspace || !ids_src)) return fail(MGR_EINVAL, "null argument");
    if (n > 0 && redirect_bin >= 0 && (!redirect_dst || !ids_redirect_dst))
        return fail(MGR_EINVAL, "redirect without buffer");
    if (redirect_bin >= nbins) return fail(MGR_EINVAL, "redirect_bin out of range");
    const mgr::Workspace ws = mgr::carve((void*)workspace, n, nbins, tile_rows);
    HIP_OK(mgr::launch_pack(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst,
                            redirect_bin, redirect_dst, (hipStream_t)stream, ids_src, ids_dst,
                            ids_redirect_dst));
    return MGR_OK;
}

int mgr_pack_tiles(const void* src, int64_t row_bytes, int64_t n, const void* dest, int nbins,
                   int drop_bin, int tile_rows, const void* workspace, void* dst, int redirect_bin,
                   void* redirect_dst, const uint16_t* ids_src, uint16_t* ids_dst,
                   uint16_t* ids_redirect_dst, int64_t tile_begin, int64_t tile_end,
                   void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (row_bytes < 1) return fail(MGR_EINVAL, "row_bytes %lld", (long long)row_bytes);
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (n > 0 && (!src || !dest || !workspace)) return fail(MGR_EINVAL, "null argument");
    if (n > 0 && redirect_bin >= 0 && (!redirect_dst || (ids_src && !ids_redirect_dst)))
        return fail(MGR_EINVAL, "redirect without buffer");
    if (redirect_bin >= nbins) return fail(MGR_EINVAL, "redirect_bin out of range");
    mgr::Workspace ws = mgr::carve((void*)workspace, n, nbins, tile_rows);
    if (tile_begin < 0 || tile_end < tile_begin || tile_end > ws.T)
        return fail(MGR_EINVAL, "tiles [%lld, %lld) of %lld", (long long)tile_begin,
                    (long long)tile_end, (long long)ws.T);
    if (tile_end == tile_begin) return MGR_OK;
    ws.t0 = tile_begin;
    ws.tn = tile_end - tile_begin;
    HIP_OK(mgr::launch_pack(src, row_bytes, n, dest, nbins, drop_bin, tile_rows, ws, dst,
                            redirect_bin, redirect_dst, (hipStream_t)stream, ids_src, ids_dst,
                            ids_redirect_dst));
    return MGR_OK;
}

int64_t mgr_onepass_workspace_bytes(int64_t n, int nbins) {
    if (n < 0 || nbins < 1 || nbins > MGR_MAX_BINS) return -1;
    return mgr::onepass_workspace_bytes(n, nbins);
}

int mgr_partition_onepass(const mgr_plan* plan, const mgr_plan* fine_plan, void* data,
                          int64_t row_bytes, int64_t pos_offset, int pos_dtype, int64_t n,
                          int periodic, void* out, uint16_t* fine_out, int64_t cap_rows,
                          int64_t* bin_counts, void* workspace, void* stream) {
    if (!plan) return fail(MGR_EINVAL, "null plan");
    if (n < 0 || cap_rows < 0) return fail(MGR_EINVAL, "n %lld, cap_rows %lld", (long long)n,
                                           (long long)cap_rows);
    if (!bin_counts || (n > 0 && (!data || !out || !workspace)))
        return fail(MGR_EINVAL, "null data/out/bin_counts/workspace");
    mgr::Geom g = plan->g;
    if (pos_dtype != MGR_F32 && pos_dtype != MGR_F64)
        return fail(MGR_EUNSUPPORTED, "one-pass partition: float32 / float64 positions only");
    pos_modes(g, pos_dtype);
    mgr::FineGeom fg;
    if (fine_plan) {
        int rc = fine_geom(plan, fine_plan, g, fg);
        if (rc) return rc;
        if (n > 0 && !fine_out) return fail(MGR_EINVAL, "fine_plan without fine_out");
    }
    const hipError_t e = mgr::launch_onepass(g, fine_plan ? &fg : nullptr, data, row_bytes,
                                             pos_offset, pos_dtype, n, periodic, out, fine_out,
                                             cap_rows, bin_counts, workspace, (hipStream_t)stream);
    if (e == hipErrorNotSupported)
        return fail(MGR_EUNSUPPORTED, "one-pass partition: shape not taken (3-D, <= 64 bins, "
                    "4-byte-multiple rows of <= 128 B holding the positions, 16-byte aligned data)");
    HIP_OK(e);
    return MGR_OK;
}

int mgr_pack_fields(int nfields, const void* const* srcs, const int64_t* row_bytes, int64_t n,
                    const void* dest, int nbins, int drop_bin, int tile_rows,
                    const void* workspace, void* const* dsts, int redirect_bin,
                    void* const* redirect_dsts, const uint16_t* ids_src, uint16_t* ids_dst,
                    uint16_t* ids_redirect_dst, int64_t tile_begin, int64_t tile_end,
                    void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (nfields < 1 || nfields > MGR_MAX_FIELDS) return fail(MGR_EINVAL, "nfields %d", nfields);
    if (!srcs || !row_bytes || !dsts) return fail(MGR_EINVAL, "null field arrays");
    if (nbins < 1 || nbins > MGR_MAX_BINS) return fail(MGR_EINVAL, "nbins %d", nbins);
    if (redirect_bin >= nbins) return fail(MGR_EINVAL, "redirect_bin out of range");
    for (int f = 0; f < nfields; ++f) {
        if (row_bytes[f] < 1) return fail(MGR_EINVAL, "field %d: row_bytes %lld", f, (long long)row_bytes[f]);
        if (n > 0 && !srcs[f]) return fail(MGR_EINVAL, "field %d: null source", f);
        if (n > 0 && redirect_bin >= 0 && (!redirect_dsts || !redirect_dsts[f]))
            return fail(MGR_EINVAL, "field %d: redirect without buffer", f);
    }
    if (n > 0 && (!dest || !workspace)) return fail(MGR_EINVAL, "null argument");
    if (n > 0 && redirect_bin >= 0 && ids_src && !ids_redirect_dst)
        return fail(MGR_EINVAL, "redirect without an ids buffer");
    if (n > 0 && ids_src && !ids_dst) return fail(MGR_EINVAL, "ids without an output");
    mgr::Workspace ws = mgr::carve((void*)workspace, n, nbins, tile_rows);
    if (tile_end >= 0) {
        if (tile_begin < 0 || tile_end < tile_begin || tile_end > ws.T)
            return fail(MGR_EINVAL, "tiles [%lld, %lld) of %lld", (long long)tile_begin,
                        (long long)tile_end, (long long)ws.T);
        if (tile_end == tile_begin) return MGR_OK;
        ws.t0 = tile_begin;
        ws.tn = tile_end - tile_begin;
    }
    HIP_OK(mgr::launch_pack_fields(nfields, srcs, row_bytes, n, dest, nbins, drop_bin, tile_rows,
                                   ws, dsts, redirect_bin, redirect_bin >= 0 ? redirect_dsts : nullptr,
                                   (hipStream_t)stream, ids_src, ids_dst, ids_redirect_dst));
    return MGR_OK;
}

int mgr_tile_offsets(const void* workspace, int64_t n, int nbins, int tile_rows,
                     const int64_t* tiles, int ntiles, int64_t* out, void* stream) {
    int rc = check_tile(tile_rows);
    if (rc) return rc;
    if (nbins < 1 || nbins > MGR_MAX_BINS || ntiles < 0 || ntiles > 4096)
        return fail(MGR_EINVAL, "nbins %d / ntiles %d", nbins, ntiles);
    if (ntiles && (!workspace || !tiles || !out)) return fail(MGR_EINVAL, "null argument");
    const mgr::Workspace ws = mgr::carve((void*)workspace, n, nbins, tile_rows);
    for (int i = 0; i < ntiles; ++i)
        if (tiles[i] < 0 || tiles[i] > ws.T) return fail(MGR_EINVAL, "tile %lld of %lld",
                                                         (long long)tiles[i], (long long)ws.T);
    if (!ntiles) return MGR_OK;
    HIP_OK(mgr::launch_tile_offsets(ws, nbins, tiles, ntiles, out, (hipStream_t)stream));
    return MGR_OK;
}

int mgr_partition_by_position(const mgr_plan* plan, void* pos, int pos_dtype, int64_t n,
                              int64_t row_stride, int periodic, const void* src,
                              int64_t row_bytes, void* dst, void* dest, int64_t* bin_counts,
                              int tile_rows, void* workspace, void* stream) {
    int rc = mgr_bin_count(plan, pos, pos_dtype, n, row_stride, periodic, dest, tile_rows,
                           workspace, stream);
    if (rc) return rc;
    rc = mgr_scan(n, plan->g.nbins, tile_rows, workspace, bin_counts, stream);
    if (rc) return rc;
    return mgr_pack(src, row_bytes, n, dest, plan->g.nbins, -1, tile_rows, workspace, dst, -1,
                    nullptr, stream);
}

// ------------------------------------------------------ halo (f1)
int mgr_halo_flags(const void* pos, int pos_dtype, int64_t n, int64_t row_stride, int dim,
                   const double* hi, const double* lo, uint16_t* flags, void* stream) {
    if (!is_pos_dtype(pos_dtype))
        return fail(MGR_EINVAL, "positions must be a float, integer or bool dtype (dtype %d)", pos_dtype);
    if (dim < 1 || dim > MGR_MAX_DIM) return fail(MGR_EINVAL, "dim %d", dim);
    if (n < 0) return fail(MGR_EINVAL, "n < 0");
    if (row_stride < dim) return fail(MGR_EINVAL, "row_stride %lld < dim %d", (long long)row_stride, dim);
    if (!hi || !lo) return fail(MGR_EINVAL, "null thresholds");
    if (n > 0 && (!pos || !flags)) return fail(MGR_EINVAL, "null argument");
    HIP_OK(mgr::launch_halo_flags(pos, pos_dtype, n, row_stride, dim, hi, lo, flags,
                                  (hipStream_t)stream));
    return MGR_OK;
}

// ------------------------------------------------------------ exchange
int mgr_comm_unique_id(void* out_id) {
    if (!out_id) return fail(MGR_EINVAL, "null id");
    ncclUniqueId id;
    NCCL_OK(ncclGetUniqueId(&id));
    static_assert(sizeof(ncclUniqueId) == MGR_UNIQUE_ID_BYTES, "unique id size");
    memcpy(out_id, &id, sizeof id);
    return MGR_OK;
}

int mgr_rccl_version(int* compiled, int* runtime) {
    if (compiled) *compiled = NCCL_VERSION_CODE;
    if (runtime) {
        int v = 0;
        NCCL_OK(ncclGetVersion(&v));
        *runtime = v;
    }
    return MGR_OK;
}

// The RCCL calls this library makes (ncclGetUniqueId, ncclCommInitRank,
// ncclSend / ncclRecv, ncclGroupStart / End, ncclAllReduce, ncclCommCount,
// ncclCommDestroy) keep their signatures and enum values throughout RCCL 2.x
// from 2.18 on; torch bundles its own RCCL (2.26 in this image) which a torch
// process has already loaded when libmgr.so binds, while the headers are
// ROCm's (2.27).  So the runtime must have the compiled major version and be
// at least kMinRccl -- anything else is refused with the two versions named,
// never run on an unmatched ABI.
static constexpr int kMinRccl = 21800;
static int rccl_check() {
    int rt = 0;
    NCCL_OK(ncclGetVersion(&rt));
    if (rt / 10000 != NCCL_VERSION_CODE / 10000 || rt < kMinRccl)
        return fail(MGR_ERCCL, "RCCL runtime %d.%d.%d is not compatible with the %d.%d.%d headers "
                    "libmgr.so was built with (needs %d.x >= %d.%d)", rt / 10000, rt / 100 % 100,
                    rt % 100, NCCL_MAJOR, NCCL_MINOR, NCCL_PATCH, NCCL_MAJOR, kMinRccl / 10000,
                    kMinRccl / 100 % 100);
    return MGR_OK;
}

int mgr_comm_create(const void* id, int nranks, int rank, mgr_comm** out) {
    if (!id || !out) return fail(MGR_EINVAL, "null argument");
    if (nranks < 1 || rank < 0 || rank >= nranks) return fail(MGR_EINVAL, "rank %d of %d", rank, nranks);
    int rc = rccl_check();
    if (rc) return rc;
    ncclUniqueId uid;
    memcpy(&uid, id, sizeof uid);
    ncclComm_t c;
    NCCL_OK(ncclCommInitRank(&c, nranks, uid, rank));
    mgr_comm* m = new mgr_comm;
    m->nccl = c;
    m->rank = rank;
    m->size = nranks;
    *out = m;
    return MGR_OK;
}

int mgr_comm_destroy(mgr_comm* comm) {
    if (!comm) return MGR_OK;
    ncclResult_t r = ncclCommDestroy(comm->nccl);
    delete comm;
    if (r != ncclSuccess) return fail(MGR_ERCCL, "ncclCommDestroy: %s", ncclGetErrorString(r));
    return MGR_OK;
}

int mgr_comm_rank(const mgr_comm* comm) { return comm ? comm->rank : -1; }
int mgr_comm_size(const mgr_comm* comm) { return comm ? comm->size : -1; }

int mgr_comm_count(const mgr_comm* comm) {
    if (!comm) return fail(MGR_EINVAL, "null comm");
    int c = 0;
    NCCL_OK(ncclCommCount(comm->nccl, &c));
    return c;
}

// An RCCL group that always closes: the first failing call inside it is
// remembered and ncclGroupEnd still runs, so a failure never leaves the
// calling thread inside an open group (later RCCL calls would misbehave).
namespace {
struct Group {
    ncclResult_t first = ncclSuccess;
    const char* what = nullptr;
    int line = 0;
    void run(ncclResult_t r, const char* expr, int ln) {
        if (r != ncclSuccess && first == ncclSuccess) {
            first = r;
            what = expr;
            line = ln;
        }
    }
    int end() {
        const ncclResult_t r = ncclGroupEnd();
        if (first != ncclSuccess)
            return fail(MGR_ERCCL, "%s: %s (%s:%d)", what, ncclGetErrorString(first), __FILE__, line);
        if (r != ncclSuccess) return fail(MGR_ERCCL, "ncclGroupEnd: %s", ncclGetErrorString(r));
        return MGR_OK;
    }
};
}  // namespace
#define GROUP_CALL(g, expr) (g).run((expr), #expr, __LINE__)

int mgr_exchange_counts(mgr_comm* comm, const int64_t* send_counts, int64_t* recv_counts,
                        void* stream) {
    return mgr_exchange_count_rows(comm, send_counts, recv_counts, 1, stream);
}

int mgr_exchange_count_rows(mgr_comm* comm, const int64_t* send, int64_t* recv, int width,
                            void* stream) {
    if (!comm || !send || !recv) return fail(MGR_EINVAL, "null argument");
    if (width < 1) return fail(MGR_EINVAL, "width %d", width);
    hipStream_t s = (hipStream_t)stream;
    NCCL_OK(ncclGroupStart());
    Group g;
    for (int p = 0; p < comm->size; ++p) {
        GROUP_CALL(g, ncclSend(send + (int64_t)p * width, (size_t)width, ncclInt64, p, comm->nccl, s));
        GROUP_CALL(g, ncclRecv(recv + (int64_t)p * width, (size_t)width, ncclInt64, p, comm->nccl, s));
    }
    return g.end();
}

// The operation list of one row exchange (what mgr_exchange_rows issues, in
// that order).  Peers are visited in ring order starting after me -- to =
// me + j, from = me - j -- so the first wave of transfers of all ranks uses
// distinct xGMI links; per peer pair the sends of one side and the receives
// of the other come in the same field order, as RCCL matches them.
int mgr_exchange_schedule(int rank, int size, int nfields, const int64_t* row_bytes,
                          const int64_t* send_counts, const int64_t* send_offsets,
                          const int64_t* recv_counts, const int64_t* recv_offsets, int skip_self,
                          mgr_xop* ops, int max_ops) {
    if (size < 1 || rank < 0 || rank >= size) return fail(MGR_EINVAL, "rank %d of %d", rank, size);
    if (nfields < 1 || !row_bytes || !send_counts || !send_offsets || !recv_counts || !recv_offsets)
        return fail(MGR_EINVAL, "null argument");
    for (int p = 0; p < size; ++p)
        if (send_counts[p] < 0 || recv_counts[p] < 0 || send_offsets[p] < 0 || recv_offsets[p] < 0)
            return fail(MGR_EINVAL, "negative count/offset for peer %d", p);
    for (int f = 0; f < nfields; ++f)
        if (row_bytes[f] < 1) return fail(MGR_EINVAL, "row_bytes[%d] = %lld", f, (long long)row_bytes[f]);
    int k = 0;
    auto put = [&](int kind, int peer, int f, int64_t src, int64_t dst, int64_t bytes) {
        if (ops && k < max_ops) ops[k] = mgr_xop{kind, peer, f, 0, src, dst, bytes};
        ++k;
    };
    for (int j = 1; j < size; ++j) {
        const int to = (rank + j) % size;
        const int from = (rank - j + size) % size;
        for (int f = 0; f < nfields; ++f) {
            const int64_t rb = row_bytes[f];
            if (send_counts[to] > 0)
                put(MGR_XOP_SEND, to, f, send_offsets[to] * rb, -1, send_counts[to] * rb);
            if (recv_counts[from] > 0)
                put(MGR_XOP_RECV, from, f, -1, recv_offsets[from] * rb, recv_counts[from] * rb);
        }
    }
    if (!skip_self && send_counts[rank] > 0) {
        if (recv_counts[rank] != send_counts[rank])
            return fail(MGR_EINVAL, "self segment: %lld rows sent, %lld expected",
                        (long long)send_counts[rank], (long long)recv_counts[rank]);
        for (int f = 0; f < nfields; ++f)
            put(MGR_XOP_COPY, rank, f, send_offsets[rank] * row_bytes[f],
                recv_offsets[rank] * row_bytes[f], send_counts[rank] * row_bytes[f]);
    }
    return k;
}

int mgr_exchange_rows(mgr_comm* comm, int nfields, const void* const* send, void* const* recv,
                      const int64_t* row_bytes, const int64_t* send_counts,
                      const int64_t* send_offsets, const int64_t* recv_counts,
                      const int64_t* recv_offsets, int skip_self, void* stream) {
    if (!comm || nfields < 1 || !send || !recv || !row_bytes || !send_counts || !send_offsets ||
        !recv_counts || !recv_offsets)
        return fail(MGR_EINVAL, "null argument");
    hipStream_t s = (hipStream_t)stream;
    const int nops = mgr_exchange_schedule(comm->rank, comm->size, nfields, row_bytes, send_counts,
                                           send_offsets, recv_counts, recv_offsets, skip_self,
                                           nullptr, 0);
    if (nops < 0) return nops;
    std::vector<mgr_xop> ops((size_t)nops);
    mgr_exchange_schedule(comm->rank, comm->size, nfields, row_bytes, send_counts, send_offsets,
                          recv_counts, recv_offsets, skip_self, ops.data(), nops);
    bool p2p = false;
    for (const mgr_xop& o : ops) p2p |= o.kind != MGR_XOP_COPY;
    if (p2p) {
        mgr::prof_begin(s, mgr::K_EXCHANGE);
        NCCL_OK(ncclGroupStart());
        Group g;
        for (const mgr_xop& o : ops) {
            if (o.kind == MGR_XOP_SEND)
                GROUP_CALL(g, ncclSend((const char*)send[o.field] + o.src_offset, (size_t)o.bytes,
                                       ncclUint8, o.peer, comm->nccl, s));
            else if (o.kind == MGR_XOP_RECV)
                GROUP_CALL(g, ncclRecv((char*)recv[o.field] + o.dst_offset, (size_t)o.bytes,
                                       ncclUint8, o.peer, comm->nccl, s));
        }
        const int rc = g.end();
        mgr::prof_end(s, mgr::K_EXCHANGE);
        if (rc) return rc;
    }
    for (const mgr_xop& o : ops)
        if (o.kind == MGR_XOP_COPY)
            HIP_OK(hipMemcpyAsync((char*)recv[o.field] + o.dst_offset,
                                  (const char*)send[o.field] + o.src_offset, (size_t)o.bytes,
                                  hipMemcpyDeviceToDevice, s));
    return MGR_OK;
}

int mgr_group_p2p(mgr_comm* comm, int nops, const int* kinds, const int* peers,
                  void* const* bufs, const int64_t* bytes, void* stream) {
    if (!comm || nops < 0 || (nops > 0 && (!kinds || !peers || !bufs || !bytes)))
        return fail(MGR_EINVAL, "null argument");
    for (int i = 0; i < nops; ++i) {
        if (kinds[i] != MGR_XOP_SEND && kinds[i] != MGR_XOP_RECV)
            return fail(MGR_EINVAL, "op %d: kind %d", i, kinds[i]);
        if (peers[i] < 0 || peers[i] >= comm->size) return fail(MGR_EINVAL, "op %d: peer %d", i, peers[i]);
        if (bytes[i] < 0 || (bytes[i] > 0 && !bufs[i])) return fail(MGR_EINVAL, "op %d: buffer", i);
    }
    hipStream_t s = (hipStream_t)stream;
    // the self pairs: the k-th send to me feeds the k-th receive from me (a
    // device copy, RCCL is not involved)
    std::vector<int> ss, rr;
    for (int i = 0; i < nops; ++i)
        if (peers[i] == comm->rank && bytes[i] > 0) (kinds[i] == MGR_XOP_SEND ? ss : rr).push_back(i);
    if (ss.size() != rr.size()) return fail(MGR_EINVAL, "self sends %zu != self receives %zu", ss.size(), rr.size());
    for (size_t k = 0; k < ss.size(); ++k) {
        if (bytes[ss[k]] != bytes[rr[k]])
            return fail(MGR_EINVAL, "self pair %zu: %lld bytes sent, %lld received", k,
                        (long long)bytes[ss[k]], (long long)bytes[rr[k]]);
        HIP_OK(hipMemcpyAsync(bufs[rr[k]], bufs[ss[k]], (size_t)bytes[ss[k]], hipMemcpyDeviceToDevice, s));
    }
    bool any = false;
    for (int i = 0; i < nops; ++i) any |= peers[i] != comm->rank && bytes[i] > 0;
    if (!any) return MGR_OK;
    mgr::prof_begin(s, mgr::K_EXCHANGE);
    NCCL_OK(ncclGroupStart());
    Group g;
    for (int i = 0; i < nops; ++i) {
        if (peers[i] == comm->rank || bytes[i] == 0) continue;
        if (kinds[i] == MGR_XOP_SEND)
            GROUP_CALL(g, ncclSend(bufs[i], (size_t)bytes[i], ncclUint8, peers[i], comm->nccl, s));
        else
            GROUP_CALL(g, ncclRecv(bufs[i], (size_t)bytes[i], ncclUint8, peers[i], comm->nccl, s));
    }
    const int rc = g.end();
    mgr::prof_end(s, mgr::K_EXCHANGE);
    return rc;
}

int mgr_comm_allreduce_max_f64(mgr_comm* comm, const double* in, double* out, int64_t count,
                               void* stream) {
    if (!comm || !in || !out || count < 0) return fail(MGR_EINVAL, "bad argument");
    NCCL_OK(ncclAllReduce(in, out, (size_t)count, ncclFloat64, ncclMax, comm->nccl,
                          (hipStream_t)stream));
    return MGR_OK;
}

// ------------------------------------------------------ synthetic data
int mgr_synth_uniform(uint64_t seed, int64_t gid0, int64_t n, int dim, const double* box,
                      double* pos, void* rec32, void* stream) {
    if (dim < 1 || dim > MGR_MAX_DIM || !box) return fail(MGR_EINVAL, "bad dim/box");
    if (rec32 && dim != 3) return fail(MGR_EINVAL, "32-byte records need dim == 3");
    if (n < 0) return fail(MGR_EINVAL, "n < 0");
    HIP_OK(mgr::launch_synth_uniform(seed, gid0, n, dim, box, pos, rec32, (hipStream_t)stream));
    return MGR_OK;
}

// ---------------------------------------------------------- test hooks
int mgr_test_hook(const char* key, int64_t value) {
    if (!key) return fail(MGR_EINVAL, "null key");
    if (mgr::set_hook(key, value))
        return fail(MGR_EINVAL, "unknown test hook '%s' or value %lld out of range", key,
                    (long long)value);
    return MGR_OK;
}

// ------------------------------------------------------------ profiler
int mgr_profile_enable(int on) {
    std::lock_guard<std::mutex> lk(mgr::g_prof_mu);
    if (!on) mgr::collect_locked();
    mgr::g_prof_on = on != 0;
    return MGR_OK;
}

int mgr_profile_reset(void) {
    std::lock_guard<std::mutex> lk(mgr::g_prof_mu);
    mgr::collect_locked();
    for (int k = 0; k < mgr::K_NUM_KERNELS; ++k) {
        mgr::g_ms[k] = 0.0;
        mgr::g_cnt[k] = 0;
    }
    return MGR_OK;
}

int mgr_profile_select(int64_t mask) {
    mgr::g_prof_mask.store(mask, std::memory_order_relaxed);
    return MGR_OK;
}

int mgr_profile_kernel_id(const char* kernel) {
    if (!kernel) return fail(MGR_EINVAL, "null kernel name");
    for (int k = 0; k < mgr::K_NUM_KERNELS; ++k)
        if (strcmp(kernel, mgr::kernel_name(k)) == 0) return k;
    return fail(MGR_EINVAL, "unknown kernel '%s'", kernel);
}

int mgr_profile_read(const char* kernel, double* total_ms, int64_t* launches) {
    if (!kernel) return fail(MGR_EINVAL, "null kernel name");
    std::lock_guard<std::mutex> lk(mgr::g_prof_mu);
    mgr::collect_locked();
    for (int k = 0; k < mgr::K_NUM_KERNELS; ++k) {
        if (strcmp(kernel, mgr::kernel_name(k)) == 0) {
            if (total_ms) *total_ms = mgr::g_ms[k];
            if (launches) *launches = mgr::g_cnt[k];
            return MGR_OK;
        }
    }
    return fail(MGR_EINVAL, "unknown kernel '%s'", kernel);
}

}  // extern "C"
