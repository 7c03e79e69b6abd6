/*
 * qldpc_decoder.h — C ABI of the MI355X (gfx950) batched BP / Min-Sum decoder.
 *
 * This is the drop-in boundary for qLDPCsim's Monte-Carlo hot path
 * (albertogp71/qLDPCsim @ 2025-12-26). The reference has no FFI: its boundary
 * is the Python call dispatched per shot by simulate_p
 * (qLDPCsim/simulator.py:270-284) into
 *     MS_decoder(H, syndrome, p, max_iter=99, layers=None, beta=0.75,
 *                OSDorder=-1, eps=1e-9) -> (e_hat int8[n], n_iter)   decoders.py:110-182
 *     BP_decoder(H, syndrome, p, max_iter=99, layers=None, OSDorder=-1,
 *                eps=1e-9) -> (e_hat int64[n], n_iter)               decoders.py:189-290
 *     OSDdec(H, e_hat, syndrome, posteriorLLRs, order=0) -> e_hat      decoders.py:299-370
 * Each entry point below names the reference interface it replaces. The
 * Python package `qldpcsim_amd` binds these with ctypes and
 * re-exposes the reference signatures unchanged.
 *
 * Conventions
 *  - Plain C types only. Every function returns QLDPC_OK (0) or a negative
 *    QLDPC_E* code; qldpc_last_error() gives a message (thread-local).
 *  - "d_" pointers are device (HBM) pointers; "h_" pointers are host memory.
 *  - `stream` is a hipStream_t passed as void* (NULL = the null stream).
 *    Device entry points are asynchronous on that stream and do no
 *    allocation, copy or synchronisation (hipGraph-capturable).
 *  - Results are bit-exact with the reference for MS (hard decisions,
 *    iteration counts, float64 posteriors) and for BP,
 *    whose tanh / arctanh / log restate the NumPy 2.2.6 / SVML functions the
 *    reference runs on the capture host (include/qldpc_libm.h); against other
 *    NumPy builds the north star's 1e-5 relative contract on BP posteriors
 *    (App. A.2) is what holds.
 */
#ifndef QLDPC_DECODER_H
#define QLDPC_DECODER_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define QLDPC_OK 0
#define QLDPC_EINVAL -1   /* bad argument / shape / option   (reference: ValueError)  */
#define QLDPC_ERANGE -2   /* index out of range               (reference: IndexError)  */
#define QLDPC_EUNSUP -3   /* graph outside the kernel's limits (degree, size, LDS)     */
#define QLDPC_EHIP -4     /* a HIP runtime call failed          (raised as RuntimeError) */
#define QLDPC_ENOMEM -5

#define QLDPC_ALGO_MS 0   /* normalized min-sum, decoders.py:110-182 */
#define QLDPC_ALGO_BP 1   /* sum-product (tanh rule), decoders.py:189-290 */

/* Bit formats of syndromes and hard decisions on the device (the *_ex entry
 * points): one byte per bit, or 64-bit words with bit j % 64 of word j / 64
 * (rows of ceil(len / 64) words; the layout of the sampler's error vectors,
 * the reference's sample row bits packed, simulator.py:246-252). */
#define QLDPC_FMT_BYTES 0
#define QLDPC_FMT_BITS 1

/* per-shot flag bits written to d_flags */
#define QLDPC_FLAG_CONVERGED 1 /* a syndrome check passed (decoders.py:175-176 / :283-285) */
#define QLDPC_FLAG_MIN_ZERO 2  /* MS: a check saw min|v|==0 (not emulated) */
#define QLDPC_FLAG_NONFINITE 4 /* BP: tanh(v/2)==0 or a non-finite message */

typedef struct qldpc_code qldpc_code;         /* Tanner graph of one H, resident in HBM */
typedef struct qldpc_schedule qldpc_schedule; /* layer partition bound to one code     */

const char *qldpc_last_error(void);
const char *qldpc_version(void);

/* Number of visible HIP devices (0 if none; never fails). */
int qldpc_device_count(void);

/* Build the Tanner graph of H (row-major uint8 m x n, entries taken mod 2,
 * as load_matrix's `(mat % 2)`, simulator.py:35; any size) and upload it to
 * the current device. Replaces the per-call `np.where(H)` edge construction of
 * BP_decoder (decoders.py:224-229) and MS_decoder's dense H masks
 * (decoders.py:148-169). */
int qldpc_code_create(const uint8_t *h_H, int m, int n, qldpc_code **out);
int qldpc_code_destroy(qldpc_code *code);
int qldpc_code_shape(const qldpc_code *code, int *m, int *n, int *n_edges);

/* Bind a layer partition to a code: layer l holds rows
 * h_layer_rows[h_layer_ptr[l] .. h_layer_ptr[l+1]). Replaces MS_decoder's /
 * BP_decoder's `layers` list (decoders.py:114, :193, consumed at :154 / :247).
 * One layer holding every row = flooding. Rows out of range -> QLDPC_ERANGE
 * (reference: IndexError at decoders.py:156 / :250). Duplicate rows inside a
 * layer are dropped (the reference's Jacobi update makes them idempotent). */
int qldpc_schedule_create(const qldpc_code *code, int n_layers, const int32_t *h_layer_ptr,
                          const int32_t *h_layer_rows, qldpc_schedule **out);
int qldpc_schedule_destroy(qldpc_schedule *sched);
/* Frees the schedule's HBM-resident-kernel workspace (grown on demand, up to
 * half of the free device memory; kept between launches otherwise), after
 * the last launch that used it has finished. The next HBM decode allocates
 * it again. */
int qldpc_schedule_release_workspace(qldpc_schedule *sched);

/* Batched decode, device pointers, asynchronous on `stream`.
 * Replaces `batch` calls of MS_decoder / BP_decoder (without the OSD
 * post-step, which the host applies to non-converged shots via
 * qldpc_osd_decode) — the inner loop of simulate_p (simulator.py:244-304).
 *   d_syn   uint8 [batch][m]   syndrome bits (0/1)
 *   p       prior error probability as passed to MS_decoder (simulate uses p/3)
 *   beta    MS normalisation (0.75 default; ignored by BP)
 *   eps     decoders.py's eps (1e-9)
 *   d_ehat  uint8 [batch][n]   hard decisions, original column order
 *   d_iters int32 [batch]      iterations as returned by the reference
 *   d_post  double[batch][n]   final posterior LLRs (nullable)
 *   d_flags int32 [batch]      QLDPC_FLAG_* (nullable)
 * Any size of H decodes: codes whose per-half-shot state fits a CU's LDS
 * (and whose tables fit 16 bits) run the LDS-resident kernels, others the
 * HBM-resident kernel (row degree <= 64), with identical results. The
 * prior L = log((1-p)/max(p, eps)) is NumPy's log (decoders.py:147, :232). */
int qldpc_decode_device(const qldpc_code *code, const qldpc_schedule *sched, int algo,
                        const uint8_t *d_syn, int64_t batch, double p, int max_iter, double beta,
                        double eps, uint8_t *d_ehat, int32_t *d_iters, double *d_post,
                        int32_t *d_flags, void *stream);

/* Name of the kernel qldpc_decode_device launches for (code, sched, algo),
 * as rocprofv3 reports it (e.g. "ms_flood_kernel<8, 4>"): lets a benchmark
 * match its live timings to a committed counter profile. No reference
 * counterpart (measurement only). */
int qldpc_decode_kernel_name(const qldpc_code *code, const qldpc_schedule *sched, int algo,
                             char *buf, int len);

/* The launch geometry of that kernel: waves per workgroup, resident
 * workgroups per CU and LDS bytes per workgroup (0, 0, 0 for the
 * HBM-resident kernel, whose geometry is fixed). Measurement only. */
int qldpc_decode_launch_info(const qldpc_code *code, const qldpc_schedule *sched, int algo,
                             int *waves_per_wg, int *wg_per_cu, int *lds_bytes);

/* qldpc_decode_device with a choice of formats: d_syn uint8 [batch][m]
 * (QLDPC_FMT_BYTES) or uint64 [batch][ceil(m/64)] (QLDPC_FMT_BITS); d_ehat
 * uint8 [batch][n] or uint64 [batch][ceil(n/64)]. Bit-packed I/O cuts the
 * kernel's HBM bytes per half-shot from m + n to 8 (ceil(m/64) + ceil(n/64)). */
int qldpc_decode_device_ex(const qldpc_code *code, const qldpc_schedule *sched, int algo, const void *d_syn,
                           int syn_format, int64_t batch, double p, int max_iter, double beta, double eps,
                           void *d_ehat, int ehat_format, int32_t *d_iters, double *d_post, int32_t *d_flags,
                           void *stream);

/* Same with host buffers: stages through page-locked host memory and device
 * memory on a stream of its own (asynchronous DMA copies, then a wait on that
 * stream only).
 * This is what the single-shot drop-in shims (MS_decoder / BP_decoder) use. */
int qldpc_decode_host(const qldpc_code *code, const qldpc_schedule *sched, int algo,
                      const uint8_t *h_syn, int64_t batch, double p, int max_iter, double beta,
                      double eps, uint8_t *h_ehat, int32_t *h_iters, double *h_post,
                      int32_t *h_flags);

/* OSD post-decoder, host. Replaces OSDdec (decoders.py:299-370) including its
 * aliasing semantics: order 0 -> solve;
 * order 1 -> flip the first information-set position, then solve;
 * order >= 2 -> identical to order 0. `h_ehat` (uint8[n]) is updated in place
 * like the reference's `e_hat[perm] = ...` (decoders.py:368).
 *   h_perm   int32[n]: np.argsort(reliability) as decoders.py:320-325 computes
 *            it (NumPy itself, or qldpc_osd_order_host).
 *   h_J / h_J_size (nullable): the complementary information set (positions
 *            in perm order, decoders.py:329-342), h_J sized n.
 *   first_info_index: position the order-1 flip applies to (infoSet[0]);
 *            -1 = emulate CPython's `list(set(range(n)) - set(J))[0]`.
 * Errors: QLDPC_ERANGE where the reference raises IndexError (the greedy basis
 * loop runs past column n-1). */
int qldpc_osd_decode(const qldpc_code *code, const uint8_t *h_syn, const int32_t *h_perm, int order,
                     uint8_t *h_ehat, int32_t *h_J, int32_t *h_J_size, int first_info_index);

/* Batched OSD over `count` shots (syn uint8[count][m], perm int32[count][n],
 * ehat uint8[count][n] in/out), `nthreads` host threads (<= 0: the process's
 * budget — affinity mask, cgroup cpu.max quota, OMP_NUM_THREADS). */
int qldpc_osd_decode_batch(const qldpc_code *code, int64_t count, const uint8_t *h_syn,
                           const int32_t *h_perm, int order, uint8_t *h_ehat, int nthreads);

/* Batched OSD on the device: one workgroup per shot, asynchronous on `stream`.
 * Same semantics as qldpc_osd_decode (orders 0, 1, >= 2) for `count` shots:
 * d_syn uint8[count][m], d_perm int32[count][n] (NumPy's reliability order),
 * d_ehat uint8[count][n] in/out, d_status int32[count] (0 ok; 1 = the
 * reference's IndexError case, e_hat left unchanged). Any size: m <= 1024 and
 * n <= 2111 run in registers / LDS, larger codes with each shot's working
 * matrix in device memory (osd_hbm_kernel; LDS holds one 64-bit word per row,
 * so m is bounded by the LDS size, about 19,000 rows: QLDPC_EUNSUP past it). */
int qldpc_osd_device(const qldpc_code *code, int64_t count, const uint8_t *d_syn,
                     const int32_t *d_perm, int order, uint8_t *d_ehat, int32_t *d_status,
                     void *stream);

/* The reliability order of decoders.py:320-325 on the device, for `count`
 * posterior rows d_post double[count][n] (n <= 2048): d_perm int32[count][n]
 * = np.argsort of the keys max(prob, 1 - prob), prob = 1/(1 + np.exp(
 * clip(post, +-100))), exactly as NumPy 2.2.6 computes them on x86-64
 * AVX512_SKX: the key through SVML's exp8_ha (include/qldpc_libm.h), the order
 * through x86-simd-sort's argsort, equal keys included (np_order.cpp states
 * the algorithm). d_tiepos[row] = n for an exact order; -1 where this order
 * leaves the row to NumPy itself (a NaN posterior, or x86-simd-sort's
 * std::sort fallback after 2 floor(log2 n) partition levels). No reference
 * counterpart as an entry point (it replaces the np.argsort call inside
 * OSDdec, decoders.py:325). */
int qldpc_osd_order_device(const qldpc_code *code, int64_t count, const double *d_post, int32_t *d_perm,
                           int32_t *d_tiepos, void *stream);

/* The same order on the host (C++, `nthreads` threads, <= 0: the process's
 * budget as qldpc_osd_decode_batch): h_perm int32[count][n],
 * h_status int32[count] = 0 exact, 1 left to NumPy (as tiepos -1 above).
 * Used to check at import that the running NumPy dispatches to the restated
 * functions (qldpcsim_amd/decoders.py), and by the host OSD path. */
int qldpc_osd_order_host(const double *h_post, int64_t count, int n, int32_t *h_perm, int32_t *h_status,
                         int nthreads);

/* x86-simd-sort's argsort (np.argsort, default kind, float64) of n keys into
 * h_perm; returns 0, or 1 for a case left to NumPy (NaN, std::sort fallback). */
int qldpc_np_argsort_host(const double *h_key, int n, int32_t *h_perm);

/* The reliability keys themselves (qldpc_osd_key), element-wise; exp_only != 0:
 * np.exp alone (SVML exp8_ha restated, |x| < 707). */
void qldpc_osd_keys_host(const double *h_post, int64_t count, double *h_key, int exp_only);

/* The restated NumPy libm (include/qldpc_libm.h: the code the BP kernels and
 * the priors run), element-wise on the host: y[i] = f(x[i]) with f = np.tanh
 * (QLDPC_LIBM_TANH, decoders.py:254), np.arctanh (QLDPC_LIBM_ATANH, :259),
 * np.log (QLDPC_LIBM_LOG, :147, :232) or np.exp (QLDPC_LIBM_EXP, :322).
 * Replaces no reference interface: it lets a caller check at run time that
 * the NumPy it runs computes the same bits (decoders.numpy_libm_pinned). */
#define QLDPC_LIBM_TANH 0
#define QLDPC_LIBM_ATANH 1
#define QLDPC_LIBM_LOG 2
#define QLDPC_LIBM_EXP 3
int qldpc_libm_eval_host(int fn, const double *h_x, int64_t count, double *h_y);

/* qldpc_osd_device with the order computed on the device
 * (qldpc_osd_order_device into the caller's workspaces d_perm / d_tiepos):
 * a shot whose order the device leaves to NumPy (tiepos -1) gets d_status 2
 * and its e_hat is left unchanged: the caller decides it with NumPy's order
 * (qldpc_osd_device). Status 0 / 1 as qldpc_osd_device. */
int qldpc_osd_device_ordered(const qldpc_code *code, int64_t count, const uint8_t *d_syn, const double *d_post,
                             int order, uint8_t *d_ehat, int32_t *d_status, int32_t *d_perm, int32_t *d_tiepos,
                             void *stream);

/* qldpc_osd_device_ordered plus a spill of the shots it leaves to the host:
 * each status-2 shot also copies its posterior row to d_spill_post[slot]
 * (double[spill_cap][n]) and its index (0 .. count-1) to d_spill_idx[slot],
 * slot = the next value of *d_spill_count (int32, zeroed by the caller), for
 * slot < spill_cap; *d_spill_count ends as the number of status-2 shots. The
 * host then fetches exactly those posteriors with one copy (no gather
 * kernel queued behind other work). */
int qldpc_osd_device_ordered_ex(const qldpc_code *code, int64_t count, const uint8_t *d_syn, const double *d_post,
                                int order, uint8_t *d_ehat, int32_t *d_status, int32_t *d_perm, int32_t *d_tiepos,
                                double *d_spill_post, int32_t *d_spill_idx, int32_t *d_spill_count,
                                int64_t spill_cap, void *stream);

/* First element of CPython's `set(range(n)) - set(J)` iteration order
 * (the reference's infoSet[0], decoders.py:344); -1 if empty. */
int qldpc_cpython_setdiff_first(int n, const int32_t *J, int nJ);

/* ---- Monte-Carlo shot source and counters on the device -----------------
 * Replace simulate_p's shot source and per-shot bookkeeping
 * (simulator.py:196-197 Stim sample, :249-252 row slicing, :291-303 outcome
 * counting) so that a batch never leaves HBM. hx / hz are the two codes of
 * the pair (same n), created on the current device.
 *
 * qldpc_channel_thresholds: the 32-bit draw thresholds of the depolarizing
 * channel, T_k = floor(k * (p/3) * 2^32) (k = 1, 2, 3); p outside [0, 1]
 * -> QLDPC_EINVAL (reference: assert at simulator.py:332).
 *
 * qldpc_channel_sample: shots shot0 .. shot0+batch-1 of the stream `seed`.
 * Per qubit j of shot s: u = Philox4x32-10(key = seed, counter = (j % 64,
 * (j / 64) / 4, s mod 2^32, s >> 32))[(j / 64) % 4]; X if u < T1, Y if
 * T1 <= u < T2, Z if T2 <= u < T3 (PAULI_CHANNEL_1(p/3,p/3,p/3),
 * simulator.py:107); errX = X|Y, errZ = Z|Y; sy_z = Hz errX mod 2,
 * sy_x = Hx errZ mod 2 (the circuit's detector layout, :249-252).
 *   d_errx, d_errz  uint64 [batch][ceil(n/64)]  bit j%64 of word j/64
 *   d_syn_z uint8 [batch][m_z],  d_syn_x uint8 [batch][m_x]
 *
 * qldpc_count_outcomes: adds this batch's outcomes to d_counters int64[6] =
 * {DecFailures_X, DecFailures_Z, decSuccessExact, decSuccessDegen,
 *  sum of iterations X, sum of iterations Z} with the reference's exact
 * definitions (simulator.py:291-303; "degen" is the integer, not mod-2,
 * product of :296-298). d_ehat_x: uint8 [batch][n] estimate of errX (the
 * decode of Hz / sy_z); d_ehat_z: estimate of errZ (Hx / sy_x); d_iters_*
 * int32 [batch]. Asynchronous on `stream`, no host synchronisation. */
int qldpc_channel_thresholds(double p, uint64_t *t1, uint64_t *t2, uint64_t *t3);
/* _ex forms: syndromes (and, for the counters, estimates) in either
 * QLDPC_FMT_* format. */
int qldpc_channel_sample_ex(const qldpc_code *hx, const qldpc_code *hz, double p, uint64_t seed,
                            uint64_t shot0, int64_t batch, uint64_t *d_errx, uint64_t *d_errz,
                            void *d_syn_z, void *d_syn_x, int syn_format, void *stream);
int qldpc_count_outcomes_ex(const qldpc_code *hx, const qldpc_code *hz, int64_t batch,
                            const uint64_t *d_errx, const uint64_t *d_errz, const void *d_syn_z,
                            const void *d_syn_x, int syn_format, const void *d_ehat_x, const void *d_ehat_z,
                            int ehat_format, const int32_t *d_iters_x, const int32_t *d_iters_z,
                            int64_t *d_counters, void *stream);
int qldpc_channel_sample(const qldpc_code *hx, const qldpc_code *hz, double p, uint64_t seed,
                         uint64_t shot0, int64_t batch, uint64_t *d_errx, uint64_t *d_errz,
                         uint8_t *d_syn_z, uint8_t *d_syn_x, void *stream);
int qldpc_count_outcomes(const qldpc_code *hx, const qldpc_code *hz, int64_t batch,
                         const uint64_t *d_errx, const uint64_t *d_errz, const uint8_t *d_syn_z,
                         const uint8_t *d_syn_x, const uint8_t *d_ehat_x, const uint8_t *d_ehat_z,
                         const int32_t *d_iters_x, const int32_t *d_iters_z, int64_t *d_counters,
                         void *stream);

/* Kernel timing (HIP events around each decode kernel launch, on the launch
 * stream). Enabled by qldpc_timing_enable(1); qldpc_timing_read returns the
 * summed kernel milliseconds and launch count since the last reset. */
int qldpc_timing_enable(int on);
int qldpc_timing_reset(void);
int qldpc_timing_read(double *total_ms, int64_t *launches);

/* Library options: which kernel family decodes, for tests (every variant is
 * checked against the oracle), A/B experiments and diagnostics. The defaults
 * are the measured best and what the product runs; the library never reads
 * the environment. A change applies from the next launch on, for every
 * schedule. Names (default):
 *   "force_hbm" (0)           every code through the HBM-resident kernel
 *   "flood_generic" (0)       flooding MS through decode_kernel, not ms_flood_kernel
 *   "layered_generic" (0)     layered MS through decode_kernel, not ms_layered_kernel
 *   "ms_lanes_per_check" (0)  layered MS: one lanes-per-check width for every layer (0: per layer)
 *   "bp_wave" (0)             BP through the one-wave decode_kernel, not the team kernels
 *   "bp_lg" (1)               layered BP: the global-table team kernel (0: tables in LDS)
 *   "bp_team_w" (0)           BP team width in waves (0: automatic)
 *   "static_sched" (0)        static half-shot striding instead of the work queue
 *   "waves_per_wg" (0), "wg_per_cu" (0)   occupancy overrides of the wave kernels
 *   "osd_column" (0)          GPU OSD through the exact-REF column kernel only
 *   "osd_tickets" (1)         GPU OSD engine wave placed by per-CU SIMD tickets
 *   "osd_prof" (0)            print per-phase OSD cycles (builds with QLDPC_OSD_TIMING)
 *   "osd_hbm" (0)             GPU OSD through the device-memory kernel at any size (tests)
 * Unknown name: QLDPC_EINVAL. */
int qldpc_set_option(const char *name, int64_t value);
int qldpc_get_option(const char *name, int64_t *value);

#ifdef __cplusplus
}
#endif
#endif /* QLDPC_DECODER_H */
