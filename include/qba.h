/*
 * qba.h -- C ABI of libqba.so, the MI355X (gfx950) engine for the data-parallel
 * core of the quantum Byzantine agreement protocol of
 * Carl0sGV/TFG---Quantum-Byzantine-Agreement (tfg.py).
 *
 * The reference has no plugin/operator API; its hot path
 * sits behind (1) the qsimov gate/executor calls and (2) four module-level
 * functions plus four inline comprehensions.  Each entry point below names
 * the reference interface it replaces.  INTEGRATION.md shows the ctypes
 * binding a maintainer of tfg.py would add.
 *
 * Conventions
 *   - Every function returns QBA_OK (0) or a negative qba_status; the message
 *     of the last failure on the calling thread is qba_last_error().  No C++
 *     exception crosses this boundary.
 *   - All array arguments named *_dev are DEVICE pointers allocated by the
 *     caller (e.g. torch tensors' data_ptr()); *_host are host pointers.
 *   - `stream` is a hipStream_t (NULL = the legacy default stream).  Work is
 *     enqueued asynchronously; functions documented as "synchronous" wait.
 *   - One qba_ctx per device; a ctx is not thread-safe (one host thread, or
 *     external locking).  The ctx owns only its scratch and compiled
 *     resource programs.
 *   - Lists are uint8 matrices lists[g][k] with row stride `ld` bytes:
 *     row g = measured group g (row 0 is what rank 1 calls Li, row 1 is Lc,
 *     row g>=2 is party g's list).  ld % 4 == 0 and the base
 *     pointer must be 4-byte aligned.
 *   - Packed lists (the *_packed entry points) hold the same matrix as NIBBLE
 *     rows: byte b of row g = value of column 2b (low nibble) | value of
 *     column 2b+1 (high nibble) << 4, row stride `ld` >= (count+1)/2 bytes
 *     (same alignment rules; a missing last column's nibble is 0).  Every
 *     sampled value is < w <= 16, so nothing is lost; the fused hot path
 *     writes half the bytes.  qba_lists_pack /
 *     qba_lists_unpack convert between the two layouts.
 *   - Count tensors are int64:  H[u][g][x] (w x (n+1) x w),
 *     C[u][g][h] ((w x (n+1) x (n+1)), symmetric, diagonal = |P_u|),
 *     P[u] = |P_u| (w).  Only Q-correlated positions (L0[k] != L1[k],
 *     tfg.py:327) are counted, binned by u = L1[k] (= Lc[k], tfg.py:182).
 */
#ifndef QBA_H
#define QBA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#if defined(__GNUC__) || defined(__clang__)
#define QBA_API __attribute__((visibility("default")))
#else
#define QBA_API
#endif

typedef struct qba_ctx qba_ctx;
typedef void *qba_stream; /* hipStream_t */

typedef enum qba_status {
  QBA_OK = 0,
  QBA_EINVAL = -1,      /* bad argument */
  QBA_EHIP = -2,        /* HIP runtime failure */
  QBA_ENOMEM = -3,      /* device allocation failed */
  QBA_EUNSUPPORTED = -4,/* outside the supported envelope (e.g. n > 15) */
  QBA_ESTATE = -5       /* e.g. no resource program compiled for this n */
} qba_status;

enum { QBA_KIND_NOTQ = 0, QBA_KIND_Q = 1 };
enum { QBA_GATE_H = 0, QBA_GATE_X = 1 }; /* gate triples: {kind, target, control|-1} */

#define QBA_MAX_PARTIES 15 /* w <= 16: one nibble per group in the 64-bit outcome */

/* ---- library / context ---------------------------------------------------------- */
QBA_API const char *qba_last_error(void);
QBA_API int qba_version(void); /* major*10000 + minor*100 + patch */
/* Nonzero when any object of this library was compiled with an experiment
 * switch (tools/exp/build.sh A/B builds, some wrong by design); 0 for the
 * shipped build. */
QBA_API int qba_build_flags(void);
QBA_API int qba_init(int device, qba_ctx **out);
QBA_API int qba_destroy(qba_ctx *ctx);
/* Pre-allocate scratch for counts launches of up to `max_blocks` workgroups so
 * that later calls never allocate (required before hipGraph capture). */
QBA_API int qba_reserve(qba_ctx *ctx, int n_parties, int64_t max_blocks);

/* ---- (A1/A2) resource preparation: dense fp64 statevector, gfx950 kernels --------- */
/* Replaces qs.QGate(...).add_operation(...) + qs.Drewom().execute(...) state
 * preparation (tfg.py:15-65, 76, 80).  Qubit 0 is the MSB of a basis index. */
QBA_API int qba_sv_init(qba_ctx *ctx, double *sv_dev, int nqubits, qba_stream stream);
QBA_API int qba_sv_apply(qba_ctx *ctx, double *sv_dev, int nqubits, const int32_t *gates_host,
                 int n_gates, qba_stream stream);
/* |0...0> followed by the gate list, in the fewest passes: single-qubit gates
 * on qubits no CX has touched yet fold into the initial product state (one
 * write-only pass), then runs of H / X / shared-control CX gates are one pass
 * each.  Same result as qba_sv_init + qba_sv_apply (tfg.py:56-65, 43-52:
 * the whole H/X layer of both circuits folds into the init pass). */
QBA_API int qba_sv_prepare(qba_ctx *ctx, double *sv_dev, int nqubits, const int32_t *gates_host,
                   int n_gates, qba_stream stream);
/* Probabilities |a_i|^2 > eps, compacted in ascending index order.  Writes at
 * most `cap` (index, prob) pairs; *count_host receives the full support size.
 * Synchronous. */
QBA_API int qba_sv_support(qba_ctx *ctx, const double *sv_dev, int nqubits, double eps,
                   int64_t *idx_dev, double *prob_dev, int64_t cap, int64_t *count_host,
                   qba_stream stream);
/* Compile one of the two circuits of an n-party run into the sampler's
 * factored alias-table program.  `gates_host` is the reference's gate list
 * for that circuit (notQCorrelated, tfg.py:15-22, or qCorrelated, tfg.py:25-40);
 * for QBA_KIND_Q, `perm_host[g-1]` is the permutation the list was built
 * with: its X gates are verified to be the classical mask the sampler draws
 * afresh per entry.  The circuit is split into entangled registers, each is
 * simulated on the device, its support compacted and turned into an alias
 * table.  Synchronous. */
QBA_API int qba_resource_compile(qba_ctx *ctx, int n_parties, int kind, const int32_t *gates_host,
                         int n_gates, const int32_t *perm_host);
/* Export the compiled program for kind (for tests / the CPU twin):
 * factor descriptors (bits, uniform, table offset, u-word) and the tables. */
QBA_API int qba_program_export(qba_ctx *ctx, int n_parties, int kind, int32_t *n_factors,
                       int32_t *desc_host /* [16][6] */, uint64_t *pat_host,
                       uint64_t *apat_host, uint64_t *thr_host, int32_t table_cap,
                       int32_t *table_len);

/* Sampler selection of the compiled pair (synchronous, host only):
 * flags[0] = canonical table layout, flags[1] = closed form (n <= 11 and both
 * programs proven equal to tfg.py's circuits' distributions), flags[2] =
 * 2^32 mod n!, flags[3..5] = permutation stage sizes A, B, C. */
QBA_API int qba_program_flags(qba_ctx *ctx, int n_parties, int32_t *flags_host /* [6] */);

/* Host only (no device needed): the closed-form permutation stage tables for
 * n in [1, 11] (layout in csrc/qba_internal.h).  sizes[0..5] = RA, RB, RC,
 * word offset of B, word offset of C, total words; `words` may be NULL to
 * query the size. */
QBA_API int qba_perm_tables(int n_parties, uint32_t *words_host, int32_t cap, int32_t *sizes_host /* [6] */);

/* ---- (A3/A4) Born sampling: Philox4x32-10 keyed by the GLOBAL entry index -------- */
/* Replaces generacionListas (tfg.py:68-84) + measure_to_ints (tfg.py:128-129):
 * writes lists[g][k - first] for entries k in [first, first+count). */
QBA_API int qba_sample(qba_ctx *ctx, int n_parties, uint64_t seed, uint64_t first, uint64_t count,
               uint8_t *lists_dev, uint64_t ld, qba_stream stream);

/* ---- (A5-A8) checks, count mode -------------------------------------------------- */
/* One pass over the lists computing H, C, P (see conventions); replaces the
 * per-packet work of tfg.py:182, 189, 291-294, 327 and consistent() 87-98 in
 * canonical order.  accumulate != 0 adds into H/C/P instead of overwriting. */
QBA_API int qba_check_counts(qba_ctx *ctx, int n_parties, const uint8_t *lists_dev, uint64_t count,
                     uint64_t ld, int64_t *H_dev, int64_t *C_dev, int64_t *P_dev,
                     int accumulate, qba_stream stream);
/* Statistics of the last counts launch on this ctx (synchronous):
 * out[0] = Q-correlated entries that held a value >= w and were therefore
 * not counted (never happens for lists from qba_sample); out[1] = workgroups
 * of an n = 11 pair-bin kernel (the fused kernel from 2^24 entries, the
 * check of nibble rows) whose 8-bit pair bins wrapped and that recounted
 * their entries exactly from the stored rows.  Pair-bin launches give a
 * workgroup at most 2^18 entries (a larger call is split, later parts
 * accumulating), where no bin wraps for sampled lists; the test seam that
 * forces wraps and pair bins on small launches (qba_test_set_knobs' list_grid
 * and pb_min_entries) gives a workgroup at most 2^23 entries per launch, below
 * group 0's 24-bit total, so a wrap is always detected exactly. */
QBA_API int qba_last_stats(qba_ctx *ctx, int64_t *out2_host);
/* Fused sample + check: lists are written once and counted from registers. */
QBA_API int qba_sample_check(qba_ctx *ctx, int n_parties, uint64_t seed, uint64_t first,
                     uint64_t count, uint8_t *lists_dev, uint64_t ld, int64_t *H_dev,
                     int64_t *C_dev, int64_t *P_dev, int accumulate, qba_stream stream);

/* The same three passes over packed (nibble-row) lists; counts identical to
 * the byte-layout calls on the same entries.  qba_check_counts_packed cannot
 * see a value > 15 (not representable); values in [w, 15] are caught as in
 * qba_check_counts (qba_last_stats).  Every counting call tests Cond3
 * (tfg.py:96-98) on every Q-correlated entry: an entry whose values are not
 * pairwise distinct adds its equal pairs to C[u][g][h]. */
QBA_API int qba_sample_packed(qba_ctx *ctx, int n_parties, uint64_t seed, uint64_t first, uint64_t count,
                              uint8_t *packed_dev, uint64_t ld, qba_stream stream);
QBA_API int qba_sample_check_packed(qba_ctx *ctx, int n_parties, uint64_t seed, uint64_t first,
                                    uint64_t count, uint8_t *packed_dev, uint64_t ld, int64_t *H_dev,
                                    int64_t *C_dev, int64_t *P_dev, int accumulate, qba_stream stream);
QBA_API int qba_check_counts_packed(qba_ctx *ctx, int n_parties, const uint8_t *packed_dev, uint64_t count,
                                    uint64_t ld, int64_t *H_dev, int64_t *C_dev, int64_t *P_dev,
                                    int accumulate, qba_stream stream);
/* Deferred reduction, for back-to-back count passes (BASELINE configs[1]:
 * sizeL = 1e6 per pass, where the separate reduce launch is a third of the
 * pass).  Same arguments and results as qba_sample_check / _packed (tfg.py:
 * 68-84, 182, 189, 291-294, 327, consistent() 87-98), but the call's H, C, P
 * and qba_last_stats are complete only after the NEXT deferred call on this
 * ctx or qba_flush_deferred(ctx): the next call's list kernel reduces this
 * call's slab rows in workgroups of its own (two alternating slab buffers),
 * dispatched after its list workgroups into the CUs they leave idle.  A
 * small call whose list workgroups fill the chip, any non-deferred counting
 * call and qba_reserve flush the pending reduction first; a pending call on
 * another stream is flushed there and ordered by an event.  A pair-bin call
 * larger than one launch's per-workgroup budget (above ~1.3e8 entries at n =
 * 11) runs its earlier parts synchronously and defers only its last part's
 * reduction; its first part flushes a pending call and then overwrites the
 * outputs, so a pending call that shares this call's H/C/P buffers ends with
 * this call's counts in them (as it would after any later call into the same
 * buffers). */
QBA_API int qba_sample_check_deferred(qba_ctx *ctx, int n_parties, uint64_t seed, uint64_t first,
                                      uint64_t count, uint8_t *lists_dev, uint64_t ld, int64_t *H_dev,
                                      int64_t *C_dev, int64_t *P_dev, int accumulate, qba_stream stream);
QBA_API int qba_sample_check_packed_deferred(qba_ctx *ctx, int n_parties, uint64_t seed, uint64_t first,
                                             uint64_t count, uint8_t *packed_dev, uint64_t ld, int64_t *H_dev,
                                             int64_t *C_dev, int64_t *P_dev, int accumulate, qba_stream stream);
/* Launches the pending deferred reduction (if any) on its call's stream.
 * Graph capture: a deferred reduction must be launched in the capture state
 * it was recorded in, so call qba_flush_deferred before beginning a capture
 * and before ending one (the deferred calls inside a capture then form a
 * closed chain).  A call that would carry a pending reduction across a
 * capture boundary fails with QBA_ESTATE; qba_flush_deferred outside the
 * capture of a captured pending reduction drops it (QBA_ESTATE: that call's
 * counts stay incomplete).  Counting calls of one ctx on different streams
 * share its scratch: a counting call on another stream than the previous
 * one synchronises the device first (so do not switch a ctx's stream while
 * another thread captures a graph on this device; qba_last_stats and
 * qba_destroy flush a pending reduction first).  Streams are told apart by
 * their handle values: synchronise a stream that ran counting calls of this
 * ctx before destroying it, since a new stream may reuse the handle.  The
 * synchronisation runs in relaxed capture mode (a graph another thread
 * captures is left alone). */
QBA_API int qba_flush_deferred(qba_ctx *ctx);
/* Rows [0, rows) of `count` columns between the layouts.  pack: *bad_dev (may
 * be NULL) receives how many values were > 15 (stored as value & 15). */
QBA_API int qba_lists_pack(qba_ctx *ctx, const uint8_t *lists_dev, uint64_t ld, int rows, uint64_t count,
                           uint8_t *packed_dev, uint64_t ldp, int64_t *bad_dev, qba_stream stream);
QBA_API int qba_lists_unpack(qba_ctx *ctx, const uint8_t *packed_dev, uint64_t ldp, int rows, uint64_t count,
                             uint8_t *lists_dev, uint64_t ld, qba_stream stream);

/* Batched independent runs (BASELINE configs[3]: 4096 independent 7-party
 * instances per GPU).  Instance i uses Philox key seed_base + i over entries
 * [0, count); its lists start at lists_dev + i*inst_stride (rows ld apart) and
 * its counts at H_dev + i*w*(n+1)*w, C_dev + i*w*(n+1)^2, P_dev + i*w. */
QBA_API int qba_sample_check_batched(qba_ctx *ctx, int n_parties, uint64_t seed_base,
                                     int64_t n_instances, uint64_t count, uint8_t *lists_dev,
                                     uint64_t ld, uint64_t inst_stride, int64_t *H_dev,
                                     int64_t *C_dev, int64_t *P_dev, qba_stream stream);

/* The same over nibble rows (ld, inst_stride in bytes of packed rows). */
QBA_API int qba_sample_check_batched_packed(qba_ctx *ctx, int n_parties, uint64_t seed_base,
                                            int64_t n_instances, uint64_t count, uint8_t *packed_dev,
                                            uint64_t ld, uint64_t inst_stride, int64_t *H_dev,
                                            int64_t *C_dev, int64_t *P_dev, qba_stream stream);

/* ---- (A5-A8) checks, exact-order mode (bit-exact protocol parity) --------------- */
/* isQCorrList = {k : Li[k] != Lc[k]} (tfg.py:327) as ascending indices.
 * *count_host receives the number found; at most `cap` are written. Synchronous. */
QBA_API int qba_isq_indices(qba_ctx *ctx, const uint8_t *li_dev, const uint8_t *lc_dev, uint64_t count,
                    int64_t *idx_dev, int64_t cap, int64_t *count_host, qba_stream stream);
/* P = {x in order : Lc[x] == v} keeping the order of `order` (tfg.py:182).
 * Every index must lie in [0, lc_len) (QBA_EINVAL otherwise; nothing outside
 * Lc is read).  Synchronous. */
QBA_API int qba_select_eq(qba_ctx *ctx, const int64_t *order_dev, int64_t m, const uint8_t *lc_dev,
                  uint64_t lc_len, int64_t v, int64_t *out_dev, int64_t *count_host, qba_stream stream);
/* Host-pointer forms of the two (the protocol host's calls; synchronous):
 * idx_host / out_host receive the selected indices.  Inputs of at most 16384
 * items run as ONE single-workgroup launch through zero-copy pinned staging
 * (no copies), larger ones through the device compaction and one D2H. */
QBA_API int qba_isq_indices_host(qba_ctx *ctx, const uint8_t *li_dev, const uint8_t *lc_dev, uint64_t count,
                                 int64_t *idx_host, int64_t cap, int64_t *count_host, qba_stream stream);
QBA_API int qba_select_eq_host(qba_ctx *ctx, const int64_t *order_host, int64_t m, const uint8_t *lc_dev,
                               uint64_t lc_len, int64_t v, int64_t *out_host, int64_t *count_host,
                               qba_stream stream);
/* tuple(Li[j] for j in P) in the given order (tfg.py:189, 291). */
QBA_API int qba_gather(qba_ctx *ctx, const uint8_t *li_dev, uint64_t list_len, const int64_t *idx_dev,
               int64_t m, int64_t *out_dev, qba_stream stream);
/* consistent(v, L, w) conditions 2 and 3 (tfg.py:93-98) over m equal-length
 * tuples stored row-major [m][len] (Cond1 and the empty-L StopIteration stay
 * on the host).  *ok_host = 1 if consistent.  Synchronous. */
QBA_API int qba_consistent(qba_ctx *ctx, const int64_t *tuples_dev, int64_t m, int64_t len, int64_t v,
                   int64_t w, int32_t *ok_host, qba_stream stream);

/* One received packet in ONE launch (tfg.py:189-192 in step 3a, 291-294 in
 * step 3b): gathers the receiver's own tuple Li[j] for j in order (its set-
 * iteration order of P) and evaluates Cond2/Cond3 of consistent(v, L | {own},
 * w) (tfg.py:93-98) over the m received tuples of length len, with the set's
 * de-duplication of own.  stage_dev = [order (len) | tuples (m x len)].
 * out_dev (len + 3 + m int64): own tuple, then bad-index flag, received-
 * tuple violation flag, own Cond2 violation flag, and per received tuple the
 * number of positions equal to own; consistent <=> all flags 0 and every
 * count in {0, len} (the host adds Cond1).  Asynchronous on `stream`. */
QBA_API int qba_check_packet(qba_ctx *ctx, const uint8_t *li_dev, uint64_t list_len,
                             const int64_t *stage_dev, int64_t m, int64_t len, int64_t v, int64_t w,
                             int64_t *out_dev, qba_stream stream);

/* Exact-order consistent(v, L, w) (tfg.py:87-98) over m tuples gathered on
 * the device (SURVEY.md §8(b) qba_check_gather): T_a[k] = lists[party[a]][
 * idx[a][k]] (lists [rows][ld], list_len valid entries per row; idx [m][len]
 * row-major).  L is a set: identical tuples collapse (tfg.py:209, 240, 260).
 * *ok_dev = 1 consistent, 0 not, -1 an index or party out of range (nothing
 * outside the lists is read).  1 <= m <= 64 (m = 0 is the reference's
 * StopIteration, tfg.py:90: QBA_EINVAL).  Asynchronous on `stream`. */
QBA_API int qba_check_gather(qba_ctx *ctx, const uint8_t *lists_dev, uint64_t ld, int rows, uint64_t list_len,
                             const int64_t *idx_dev, const int32_t *party_dev, int64_t m, int64_t len,
                             int64_t v, int64_t w, int32_t *ok_dev, qba_stream stream);

/* Synchronous host-pointer form of qba_check_packet (the protocol's
 * per-packet call: one H2D through the context's pinned staging, one launch,
 * one D2H, one sync).  stage_host / out_host as above, in host memory. */
QBA_API int qba_check_packet_host(qba_ctx *ctx, const uint8_t *li_dev, uint64_t list_len,
                                  const int64_t *stage_host, int64_t m, int64_t len, int64_t v, int64_t w,
                                  int64_t *out_host, qba_stream stream);

/* A whole round of received packets (tfg.py:337-348 -> 289-294) in ONE host
 * round trip: k stages concatenated in stage_host (packet i: len_i*(m_i+1)
 * int64 = [order | rows], desc[i] = {m_i, len_i, v_i}); out_host receives the
 * k outputs concatenated (packet i: len_i + 3 + m_i int64, as
 * qba_check_packet).  One H2D, k launches, one D2H, one sync. */
QBA_API int qba_check_packets_host(qba_ctx *ctx, const uint8_t *li_dev, uint64_t list_len,
                                   const int64_t *stage_host, const int64_t *desc, int64_t k, int64_t w,
                                   int64_t *out_host, qba_stream stream);

/* ---- host-only: the exact-order protocol's set semantics (no device) -------------- */
/* Iteration order of CPython 3.10's set(keys) for int64 keys inserted in the
 * given order (tfg.py:240 P = set(buff); tfg.py:182 and 327 set
 * comprehensions): order_out[*n_out] = the distinct keys in slot order.
 * Replaces building the Python set and reading it back (tfg.py:189, 209, 291
 * iterate it).  order_out needs room for n keys. */
QBA_API int qba_host_pyset_order(const int64_t *keys, int64_t n, int64_t *order_out, int64_t *n_out);
/* hash(tuple(vals)) of CPython 3.10 (tuplehash over int elements): the set of
 * tuples L (tfg.py:189, 260, 291) orders and de-duplicates by it. */
QBA_API int qba_host_pytuple_hash(const int64_t *vals, int64_t n, int64_t *hash_out);

/* ---- wire-compatible codec (rawS layout, tfg.py:81-84, 128-129, 142-161) -------- */
QBA_API int qba_bits_to_values(qba_ctx *ctx, const int64_t *raw_dev, uint64_t count, int nq,
                       uint8_t *values_dev, qba_stream stream);
QBA_API int qba_values_to_bits(qba_ctx *ctx, const uint8_t *values_dev, uint64_t count, int nq,
                       int64_t *raw_dev, qba_stream stream);
/* rawS of a run (tfg.py:81-84, as rank 0 ships it at tfg.py:142-145): rows
 * [0, rows) of a lists matrix encoded to raw_host[rows][count*nq].  Sync. */
QBA_API int qba_lists_to_bits_host(qba_ctx *ctx, const uint8_t *lists_dev, uint64_t ld, int rows,
                                   uint64_t count, int nq, int64_t *raw_host, qba_stream stream);
/* measure_to_ints of a received row (tfg.py:158, 161) straight from the
 * receive buffer in host memory to a device list.  raw_host may be reused
 * as soon as the call returns; the decode is ordered on `stream` (small rows
 * are read from zero-copy staging without waiting; larger ones wait). */
QBA_API int qba_bits_to_values_host(qba_ctx *ctx, const int64_t *raw_host, uint64_t count, int nq,
                                    uint8_t *values_dev, qba_stream stream);

/* ---- multi-GPU: the count all-reduce over RCCL ---------------- */
/* The sizeL shards of one run live on G GPU-owner ranks; their int64 count
 * buffers [H | C | P] are summed with ONE all-reduce.  This replaces nothing
 * in tfg.py (the reference is single-process per party and never shards a
 * list); it is what a non-torch caller (the mpiexec host) uses where the
 * torch path calls torch.distributed.all_reduce.  Bootstrap: rank 0 calls
 * qba_rccl_unique_id, ships the 128 bytes to the other owners (e.g. over
 * MPI), every owner calls qba_rccl_init.  librccl is opened on first use;
 * QBA_EUNSUPPORTED without it. */
QBA_API int qba_rccl_unique_id(uint8_t *id_host /* [128] */);
QBA_API int qba_rccl_init(qba_ctx *ctx, const uint8_t *id_host, int nranks, int rank);
/* In place, sum over the communicator's ranks; asynchronous on `stream`. */
QBA_API int qba_allreduce_i64(qba_ctx *ctx, int64_t *buf_dev, int64_t count, qba_stream stream);

/* ---- helpers exported for tests ------------------------------------------------- */
/* Vose alias table over k probabilities (host): thr[i] in [0, 2^32] (2^32 =
 * always keep column i), alias[i] = column taken otherwise. */
QBA_API int qba_alias_build(const double *prob_host, int32_t k, uint64_t *thr_host, int32_t *alias_host);
/* Philox4x32-10 on the device for KATs: out[4*i..] = philox(ctr_i, key). */
QBA_API int qba_philox_dev(qba_ctx *ctx, const uint32_t *ctr_dev, int64_t n, uint64_t key,
                   uint32_t *out_dev, qba_stream stream);
/* Test seam: the launch-shape knobs the GPU tests use to reach the list
 * kernels' rare paths on small inputs (the library reads no environment
 * variable).  chunk_entries: entries per list-kernel launch (0 = the shipped
 * 2^31; else 4 .. 2^31, rounded down to a multiple of 4) -- chunk splits;
 * pb_min_entries: launches from this many entries count n = 11 in pair bins
 * (< 0 = the shipped 2^24); list_grid: > 0 caps the list kernels' workgroups
 * and forces pair bins, each workgroup taking up to 2^23 entries per launch
 * -- pair-bin wraps and their recount (0 = off).  Flushes a pending deferred
 * reduction first.  Results are bit-identical under every setting. */
QBA_API int qba_test_set_knobs(qba_ctx *ctx, uint64_t chunk_entries, int64_t pb_min_entries, int list_grid);

#ifdef __cplusplus
}
#endif
#endif /* QBA_H */
