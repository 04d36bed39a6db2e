// qba_sv.hip -- dense real-fp64 statevector kernels for the resource state
// (tfg.py:15-65).  H, X and controlled-X keep amplitudes real, so a state of
// q qubits is 2^q doubles (8 B each; 2^35 = 275 GB is the largest that fits
// one MI355X).  Qubit 0 is the most significant bit of the basis index.
//
// Gate fusion (each pass is one streaming read+write of the state, so the
// cost of a circuit is its number of passes):
//  * single-qubit gates that act on a qubit before any CX touches it commute
//    to the front and fold into the initial state: |0...0> followed by them
//    is a product state written in ONE write-only pass (qba_k_sv_product);
//    tfg.py's two circuits are entirely H/X layers followed by CX gates, so
//    their whole single-qubit layer costs nothing beyond the init pass;
//  * a run of H gates (distinct qubits commute; two H on one qubit cancel)
//    is one Walsh-Hadamard pass over up to QBA_HSET_MAX bits per pass
//    (qba_k_sv_hset: each thread owns the 2^K amplitudes of one coset);
//  * a window of pairwise-commuting X / CX gates is one XOR pass: a single
//    control (or none) -> qba_k_sv_xmask, several -> qba_k_sv_xmulti.
// Threads access 16 B (a double2) whenever bit 0 lets them, and a wave's
// access covers contiguous bytes (half-dense only when bits 0 and 1 are both
// in an H set), so each pass is bound by HBM at 16 B of traffic per amplitude
// it moves (8 read + 8 written; the product pass writes 8 B per amplitude and
// reads nothing); the streaming passes use nontemporal accesses.
#include "qba_compact.h"

static constexpr double kInvSqrt2 = 0.70710678118654752440;
#define QBA_HSET_MAX 5

__device__ __forceinline__ uint64_t qba_ins0(uint64_t i, int b) {  // insert a 0 bit at position b
  const uint64_t lo = i & ((1ull << b) - 1ull);
  return ((i >> b) << (b + 1)) | lo;
}

typedef double qba_d2v __attribute__((ext_vector_type(2)));
__device__ __forceinline__ double2 qba_ld(const double2 *p, bool nt) {
  if (!nt) return *p;
  const qba_d2v v = __builtin_nontemporal_load(reinterpret_cast<const qba_d2v *>(p));
  return make_double2(v.x, v.y);
}
__device__ __forceinline__ void qba_st(double2 *p, double2 v, bool nt) {
  if (!nt) {
    *p = v;
    return;
  }
  qba_d2v w;
  w.x = v.x;
  w.y = v.y;
  __builtin_nontemporal_store(w, reinterpret_cast<qba_d2v *>(p));
}

// amplitude(i) = scale * (-1)^popcount(i & minus) if (i & fixmask) == fixval,
// else 0: |0...0> after any H/X gates on distinct untouched qubits (a fixed
// qubit is |0> or |1>; a superposed one |+> or |-> with its sign in `minus`)
__global__ void qba_k_sv_product(double2 *__restrict__ sv, uint64_t n2, uint64_t fixmask, uint64_t fixval,
                                 uint64_t minus, double scale) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n2;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = 2 * t;
    double v[2];
#pragma unroll
    for (int k = 0; k < 2; ++k) {
      const uint64_t ik = i + k;
      const double sg = (__popcll(ik & minus) & 1) ? -scale : scale;
      v[k] = ((ik & fixmask) == fixval) ? sg : 0.0;
    }
    qba_st(sv + t, make_double2(v[0], v[1]), true);
  }
}

struct QbaHBits {
  int b[QBA_HSET_MAX];        // bit positions, ascending
  uint64_t bit[QBA_HSET_MAX]; // 1 << b[j]
  double scale;               // 2^(-K/2)
};

// H on K qubits at once: the 2^K amplitudes of the coset base | span(bits)
// get a K-stage Walsh-Hadamard butterfly in registers.  V: bit 0 is in the
// set, so pairs (m, m|1) are one double2 access.
template <int K, bool V>
__global__ void qba_k_sv_hset(double *__restrict__ sv, QbaHBits hb, uint64_t nthreads) {
  constexpr int M = 1 << K;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads;
       t += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t base = t;
#pragma unroll
    for (int j = 0; j < K; ++j) base = qba_ins0(base, hb.b[j]);
    double a[M];
#pragma unroll
    for (int m = 0; m < M; m += (V ? 2 : 1)) {
      uint64_t off = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if ((m >> j) & 1) off |= hb.bit[j];
      if (V) {
        const double2 x = *reinterpret_cast<const double2 *>(sv + (base | off));
        a[m] = x.x;
        a[m + 1] = x.y;
      } else {
        a[m] = sv[base | off];
      }
    }
#pragma unroll
    for (int j = 0; j < K; ++j)
#pragma unroll
      for (int m = 0; m < M; ++m)
        if (!((m >> j) & 1)) {
          const double x = a[m], y = a[m | (1 << j)];
          a[m] = x + y;
          a[m | (1 << j)] = x - y;
        }
#pragma unroll
    for (int m = 0; m < M; m += (V ? 2 : 1)) {
      uint64_t off = 0;
#pragma unroll
      for (int j = 0; j < K; ++j)
        if ((m >> j) & 1) off |= hb.bit[j];
      if (V)
        *reinterpret_cast<double2 *>(sv + (base | off)) = make_double2(a[m] * hb.scale, a[m + 1] * hb.scale);
      else
        sv[base | off] = a[m] * hb.scale;
    }
  }
}

// XOR-mask permutation, optionally controlled: every index i with the
// control bit set (bc < 0: every index) swaps amplitudes with i ^ M.  One
// controlled X is M = 1 << bt; a run of CX gates sharing a control (they
// commute: all targets differ from the control) or a run of X gates is the
// XOR of their target bits, so a whole run costs one pass (the Q resource's
// GHZ register: n CX gates from qubit 0 -> one pass, tfg.py:38-39).
// Threads enumerate the pair representatives (bit brep = the HIGHEST bit of
// M clear, control bit set), two adjacent indices (i, i+1) per thread with
// double2 accesses when neither brep nor the control is bit 0.  The partner
// of that pair is (i^M, (i+1)^M): the aligned double2 at i^M when bit 0 is
// not in M, else the one at (i+1)^M = (i^M) - 1 with its halves swapped.
// Consecutive threads therefore touch contiguous bytes on both sides even
// when M holds low bits (they only mirror the order inside a block).
template <bool NT>
__global__ void qba_k_sv_xmask(double *__restrict__ sv, int bc, int brep, uint64_t M, uint64_t nthreads,
                               int vec) {
  const int blo = (bc >= 0 && bc < brep) ? bc : brep, bhi = (bc >= 0 && bc < brep) ? brep : bc;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads;
       t += (uint64_t)gridDim.x * blockDim.x) {
    uint64_t i = vec ? 2 * t : t;
    i = qba_ins0(i, blo);
    if (bc >= 0) i = qba_ins0(i, bhi) | (1ull << bc);
    const uint64_t j = i ^ M;
    if (vec) {
      double2 *p0 = reinterpret_cast<double2 *>(sv + i);
      double2 *p1 = reinterpret_cast<double2 *>(sv + ((M & 1ull) ? j - 1 : j));
      const double2 a = qba_ld(p0, NT), c = qba_ld(p1, NT);
      if (M & 1ull) {
        qba_st(p0, make_double2(c.y, c.x), NT);
        qba_st(p1, make_double2(a.y, a.x), NT);
      } else {
        qba_st(p0, c, NT);
        qba_st(p1, a, NT);
      }
    } else {
      const double a = sv[i];
      sv[i] = sv[j];
      sv[j] = a;
    }
  }
}

// Several commuting X / CX runs in ONE pass.  Within a window of CX gates in
// which no gate's target is another's control, every control bit is left
// unchanged by all of them, so the window is the involution i <-> i ^ M(i),
// M(i) = m0 ^ (XOR of cmask[k] over the controls k set in i).  Each index is
// visited by the lower index of its pair (the other lane of the pair idles);
// with no control on bit 0, (i, i+1) share M and move as one double2 (the
// partner double2 halves swapped when bit 0 is in M).  tfg.py:38-39's CX
// layer (controls 0..nq-1 fanned out to every group) is one such pass.
#define QBA_XRUN_MAX 8
struct QbaXRuns {
  int n;
  int cbit[QBA_XRUN_MAX];
  uint64_t cmask[QBA_XRUN_MAX];
  uint64_t m0;
};

__global__ void qba_k_sv_xmulti(double *__restrict__ sv, QbaXRuns r, uint64_t nthreads, int vec) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads;
       t += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t i = vec ? 2 * t : t;
    uint64_t M = r.m0;
    for (int k = 0; k < r.n; ++k)
      if ((i >> r.cbit[k]) & 1ull) M ^= r.cmask[k];
    if (M == 0) continue;
    const uint64_t j = i ^ M;
    if (vec) {
      const uint64_t jb = j & ~1ull;
      if (jb < i) continue;
      double2 *p0 = reinterpret_cast<double2 *>(sv + i), *p1 = reinterpret_cast<double2 *>(sv + jb);
      const double2 a = *p0, c = *p1;
      if (M & 1ull) {
        *p0 = make_double2(c.y, c.x);
        *p1 = make_double2(a.y, a.x);
      } else {
        *p0 = c;
        *p1 = a;
      }
    } else {
      if (j < i) continue;
      const double a = sv[i];
      sv[i] = sv[j];
      sv[j] = a;
    }
  }
}

static unsigned sv_grid(uint64_t nthreads) {
  uint64_t g = (nthreads + 255) / 256;
  return (unsigned)(g > 65536 ? 65536 : (g < 1 ? 1 : g));
}

static int sv_check_gates(const char *who, int nq, const int32_t *gates, int ngates) {
  for (int g = 0; g < ngates; ++g) {  // validate everything before launching anything
    const int32_t k = gates[3 * g], t = gates[3 * g + 1], c = gates[3 * g + 2];
    if ((k != QBA_GATE_H && k != QBA_GATE_X) || t < 0 || t >= nq || c >= nq || c == t ||
        (c < -1) || (k == QBA_GATE_H && c >= 0))
      return qba_fail(QBA_EINVAL, std::string(who) + ": gate " + std::to_string(g) + " is invalid");
  }
  return QBA_OK;
}

static int sv_launch_product(double *sv, int nq, uint64_t fixmask, uint64_t fixval, uint64_t minus, double scale,
                             hipStream_t s) {
  const uint64_t n2 = 1ull << (nq - 1);
  hipLaunchKernelGGL(qba_k_sv_product, dim3(sv_grid(n2)), dim3(256), 0, s, reinterpret_cast<double2 *>(sv), n2,
                     fixmask, fixval, minus, scale);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

template <int K>
static void sv_launch_hset_k(double *sv, const QbaHBits &hb, uint64_t nthr, hipStream_t s) {
  if (hb.b[0] == 0)
    hipLaunchKernelGGL((qba_k_sv_hset<K, true>), dim3(sv_grid(nthr)), dim3(256), 0, s, sv, hb, nthr);
  else
    hipLaunchKernelGGL((qba_k_sv_hset<K, false>), dim3(sv_grid(nthr)), dim3(256), 0, s, sv, hb, nthr);
}

// H on every bit of `mask`: ceil(popcount / QBA_HSET_MAX) Walsh-Hadamard passes
static int sv_launch_hset(double *sv, int nq, uint64_t mask, hipStream_t s) {
  while (mask) {
    QbaHBits hb{};
    int k = 0;
    while (mask && k < QBA_HSET_MAX && k < nq) {
      const int b = __builtin_ctzll(mask);
      mask &= mask - 1;
      hb.b[k] = b;
      hb.bit[k] = 1ull << b;
      ++k;
    }
    hb.scale = std::ldexp(1.0, -(k / 2)) * ((k & 1) ? kInvSqrt2 : 1.0);
    const uint64_t nthr = (1ull << nq) >> k;
    switch (k) {
      case 1: sv_launch_hset_k<1>(sv, hb, nthr, s); break;
      case 2: sv_launch_hset_k<2>(sv, hb, nthr, s); break;
      case 3: sv_launch_hset_k<3>(sv, hb, nthr, s); break;
      case 4: sv_launch_hset_k<4>(sv, hb, nthr, s); break;
      default: sv_launch_hset_k<5>(sv, hb, nthr, s); break;
    }
    QBA_HIP(hipGetLastError());
  }
  return QBA_OK;
}

// the fused pass sequence of an (already validated) gate list
static int sv_apply_fused(double *sv, int nq, const int32_t *gates, int ngates, hipStream_t s) {
  // X / CX gates accumulate into a window of commuting runs (one run per
  // control, ctl -1 = uncontrolled X) flushed as ONE pass; H gates into a
  // Walsh-Hadamard set (H H = I).  A gate that does not commute with the
  // open window (its target is a window control, or its control a window
  // target) or a ninth control closes the window.
  int nrun = 0;
  int run_bc[QBA_XRUN_MAX];
  uint64_t run_mask[QBA_XRUN_MAX], m0 = 0, ctl_bits = 0, tgt_bits = 0, h_mask = 0;
  auto flush_x = [&]() -> int {
    QbaXRuns r{};
    for (int k = 0; k < nrun; ++k)
      if (run_mask[k]) {
        r.cbit[r.n] = run_bc[k];
        r.cmask[r.n++] = run_mask[k];
      }
    r.m0 = m0;
    nrun = 0;
    m0 = ctl_bits = tgt_bits = 0;
    if (r.n == 0 && r.m0 == 0) return QBA_OK;
    if (r.n + (r.m0 ? 1 : 0) == 1) {  // a single run: pair representatives only
      const int bc = r.n ? r.cbit[0] : -1;
      const uint64_t M = r.n ? r.cmask[0] : r.m0;
      const int brep = 63 - __builtin_clzll(M);
      const int vec = (brep != 0 && bc != 0 && nq >= (bc >= 0 ? 3 : 2)) ? 1 : 0;
      const uint64_t npairs = (1ull << (nq - 1)) >> (bc >= 0 ? 1 : 0);
      const uint64_t nthr = npairs / (vec ? 2 : 1);
      // nontemporal: the pass streams each line once (+2%: profiles/r2/ab11_sv_nontemporal.txt)
      hipLaunchKernelGGL(qba_k_sv_xmask<true>, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, bc, brep, M, nthr, vec);
    } else {
      bool vec = nq >= 2;
      for (int k = 0; k < r.n; ++k) vec = vec && r.cbit[k] != 0;
      const uint64_t nthr = (1ull << nq) >> (vec ? 1 : 0);
      hipLaunchKernelGGL(qba_k_sv_xmulti, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, r, nthr, vec ? 1 : 0);
    }
    QBA_HIP(hipGetLastError());
    return QBA_OK;
  };
  auto flush_h = [&]() -> int {
    const uint64_t m = h_mask;
    h_mask = 0;
    return m ? sv_launch_hset(sv, nq, m, s) : QBA_OK;
  };
  for (int g = 0; g < ngates; ++g) {
    const int32_t k = gates[3 * g], t = gates[3 * g + 1], c = gates[3 * g + 2];
    const int bt = nq - 1 - t;
    if (k == QBA_GATE_X) {
      if (int e = flush_h()) return e;
      const int bc = c < 0 ? -1 : nq - 1 - c;
      int slot = -1;
      for (int q = 0; q < nrun; ++q)
        if (run_bc[q] == bc) slot = q;
      const bool commutes = !((ctl_bits >> bt) & 1ull) && (bc < 0 || !((tgt_bits >> bc) & 1ull));
      if (!commutes || (bc >= 0 && slot < 0 && nrun == QBA_XRUN_MAX)) {
        if (int e = flush_x()) return e;
        slot = -1;
      }
      tgt_bits |= 1ull << bt;
      if (bc < 0) {
        m0 ^= 1ull << bt;
        continue;
      }
      if (slot < 0) {
        slot = nrun++;
        run_bc[slot] = bc;
        run_mask[slot] = 0;
      }
      run_mask[slot] ^= 1ull << bt;
      ctl_bits |= 1ull << bc;
      continue;
    }
    if (int e = flush_x()) return e;
    h_mask ^= 1ull << bt;  // H H = I
  }
  if (int e = flush_x()) return e;
  return flush_h();
}

extern "C" int qba_sv_init(qba_ctx *ctx, double *sv, int nq, qba_stream stream) {
  if (!ctx || !sv || nq < 1 || nq > 40) return qba_fail(QBA_EINVAL, "qba_sv_init: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const uint64_t all = nq == 64 ? ~0ull : ((1ull << nq) - 1ull);
  return sv_launch_product(sv, nq, all, 0, 0, 1.0, (hipStream_t)stream);
}

extern "C" int qba_sv_apply(qba_ctx *ctx, double *sv, int nq, const int32_t *gates, int ngates,
                            qba_stream stream) {
  if (!ctx || !sv || nq < 1 || nq > 40 || ngates < 0 || (ngates && !gates))
    return qba_fail(QBA_EINVAL, "qba_sv_apply: bad arguments");
  int rc = sv_check_gates("qba_sv_apply", nq, gates, ngates);
  if (rc) return rc;
  if ((rc = qba_set_device(ctx))) return rc;
  return sv_apply_fused(sv, nq, gates, ngates, (hipStream_t)stream);
}

// |0...0> then the gate list.  Single-qubit gates on qubits no CX has touched
// yet commute with every earlier kept gate (those act on touched qubits
// only), so they are folded into the initial product state; each qubit's
// state stays one of |0>, |1>, |+>, |-> up to a sign, tracked exactly.
extern "C" int qba_sv_prepare(qba_ctx *ctx, double *sv, int nq, const int32_t *gates, int ngates,
                              qba_stream stream) {
  if (!ctx || !sv || nq < 1 || nq > 40 || ngates < 0 || (ngates && !gates))
    return qba_fail(QBA_EINVAL, "qba_sv_prepare: bad arguments");
  int rc = sv_check_gates("qba_sv_prepare", nq, gates, ngates);
  if (rc) return rc;
  if ((rc = qba_set_device(ctx))) return rc;
  // per qubit: sup = superposed; fixed: bit v, sign s0; superposed: amplitude
  // signs (s0, s1) of |0>, |1> (magnitude 1/sqrt2 each)
  std::vector<char> touched(nq, 0), sup(nq, 0), v(nq, 0);
  std::vector<int> s0(nq, 1), s1(nq, 1);
  std::vector<int32_t> rest;
  rest.reserve(3 * (size_t)ngates);
  for (int g = 0; g < ngates; ++g) {
    const int32_t k = gates[3 * g], t = gates[3 * g + 1], c = gates[3 * g + 2];
    if (c >= 0 || touched[t]) {
      if (c >= 0) touched[c] = 1;
      touched[t] = 1;
      rest.insert(rest.end(), {k, t, c});
      continue;
    }
    if (k == QBA_GATE_X) {
      if (sup[t]) std::swap(s0[t], s1[t]);
      else v[t] ^= 1;
    } else if (!sup[t]) {  // H (s|v>) = s (|0> + (-1)^v |1>) / sqrt2
      sup[t] = 1;
      s1[t] = v[t] ? -s0[t] : s0[t];
    } else {  // H (s0|0> + s1|1>)/sqrt2 = s0|0> if s0 == s1, else s0|1>
      sup[t] = 0;
      v[t] = s0[t] == s1[t] ? 0 : 1;
    }
  }
  uint64_t fixmask = 0, fixval = 0, minus = 0;
  int nsup = 0, sign = 1;
  for (int q = 0; q < nq; ++q) {
    const uint64_t bit = 1ull << (nq - 1 - q);
    sign *= s0[q];
    if (sup[q]) {
      ++nsup;
      if (s0[q] != s1[q]) minus |= bit;
    } else {
      fixmask |= bit;
      if (v[q]) fixval |= bit;
    }
  }
  const double scale = sign * std::ldexp(1.0, -(nsup / 2)) * ((nsup & 1) ? kInvSqrt2 : 1.0);
  if ((rc = sv_launch_product(sv, nq, fixmask, fixval, minus, scale, (hipStream_t)stream))) return rc;
  return sv_apply_fused(sv, nq, rest.data(), (int)rest.size() / 3, (hipStream_t)stream);
}

struct QbaSupportPred {
  const double *sv;
  double eps;
  int64_t *idx;
  double *prob;
  __device__ bool test(int64_t i) const { return sv[i] * sv[i] > eps; }
  __device__ void emit(int64_t i, int64_t pos) const {
    idx[pos] = i;
    prob[pos] = sv[i] * sv[i];
  }
};

extern "C" int qba_sv_support(qba_ctx *ctx, const double *sv, int nq, double eps, int64_t *idx,
                              double *prob, int64_t cap, int64_t *count_host, qba_stream stream) {
  if (!ctx || !sv || !count_host || nq < 1 || nq > 40 || cap < 0 || (cap && (!idx || !prob)))
    return qba_fail(QBA_EINVAL, "qba_sv_support: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  return qba_compact(ctx, QbaSupportPred{sv, eps, idx, prob}, (int64_t)1 << nq, cap, count_host,
                     (hipStream_t)stream);
}
