/* libmgr.so instrumentation: measurement and test hooks.
 *
 * NOT part of the drop-in boundary (include/mgr.h): nothing here changes what
 * the library computes.  bench.py uses the profiler to time kernels with HIP
 * events inside its timed region; the parity tests use the hooks to make a
 * fallback path run on inputs that would not take it.
 */
#ifndef MGR_INSTRUMENT_H_
#define MGR_INSTRUMENT_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---------------------------------------------------------- test hooks --
 * Force a product-reachable fallback or tile shape (results unchanged):
 * "tile_rounds" (0 = automatic, else rows per tile / 64), "scan_chunk" and
 * "scan_max_chunks" (one-pass scan chunking), "scan_spins" (polls per
 * look-back word before the scan gives up; -1 gives up at once: the failure
 * path), "pack_img_all" (image pack for 12..60-byte rows, not only 24..60),
 * "rank_rows" (0 / 2048 / 4096 ranked fine-sort tiles), "bin_unstaged" (bin
 * kernel without LDS slab staging), "bin_generic" (bin kernel with run-time
 * geometry for simple plans), "pack_generic" (the wave-per-tile pack for <= 64
 * bins), "scan_delay_bin" / "scan_delay_sleeps" (the scan chunk that ends
 * that bin counts itself done, then sleeps that many s_sleep(127) before
 * storing its inclusive word: the visibility order relaxed atomics on two
 * words allow, forced) and "scan_end_spins" (polls of the bin-end words by
 * the scan's last chunk, -1 = scan_spins; 0 = one look, which then reports
 * the forced race as a failed scan), "scan_poison_chunk" (the scan chunk with
 * this ticket publishes its prefix poisoned: a deterministic failed scan,
 * -1 = none), "fields_kernel" (multi-field packs: 0 the product's choice,
 * 1 the per-wave LDS-image kernel, 2 the tile-image kernel, 3 the
 * cooperative kernel -- each where it takes the fields, else the next).
 * Each call publishes a new immutable
 * snapshot of every hook (the library's launches read one snapshot each);
 * < 0 for an unknown key or an out-of-range value.                         */
int mgr_test_hook(const char* key, int64_t value);
/* The element types a plan computes in for positions of pos_dtype and a box
 * of box_dtype (mgr_dtype codes): *wrap = numpy's type of position % box,
 * *quot = of position / box (the bin's division), from the library's own
 * promotion table.  Host only, no GPU: tests/test_capi.py checks every pair
 * against numpy.  MGR_EINVAL for an unknown code.                          */
int mgr_test_pos_modes(int pos_dtype, int box_dtype, int* wrap, int* quot);

/* ----------------------------------------------------------- profiling --
 * Per-kernel HIP-event timing of every launch made while enabled, on the
 * launch's own stream.  mgr_profile_read synchronises those events and
 * returns the accumulated device time (ms) and launch count of the named
 * kernel ("bin_count", "scan", "pack", "cell_ids", "bin_ids", "cellnum_idx",
 * "synth", "halo" (mgr_halo_flags, mgr_msel_count), "bin_fine"
 * (mgr_bin_count_fine), "count_ids" (mgr_count_ids, mgr_rank_ids),
 * "pack_fine" (the 65..1024-bin and ranked packs), "pack_narrow" (rows < 4
 * bytes), "halo_pack" (mgr_msel_pack*)) or of the RCCL grouped row exchange
 * ("exchange").  mgr_profile_select: bit k of mask times kernel id k
 * (mgr_profile_kernel_id), default all.                                    */
int mgr_profile_enable(int on);
int mgr_profile_reset(void);
int mgr_profile_select(int64_t mask);
int mgr_profile_read(const char* kernel, double* total_ms, int64_t* launches);
int mgr_profile_kernel_id(const char* kernel);

#ifdef __cplusplus
}
#endif
#endif /* MGR_INSTRUMENT_H_ */
