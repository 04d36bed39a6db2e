// qba_sv.hip -- dense real-fp64 statevector kernels for the resource state
// (tfg.py:15-65).  H, X and controlled-X keep amplitudes real, so a state of
// q qubits is 2^q doubles (8 B each; 2^35 = 275 GB is the largest that fits
// one MI355X).  Qubit 0 is the most significant bit of the basis index.
//
// Every H gate is one streaming pass over the state, and every RUN of X
// gates or of CX gates sharing a control is one XOR-mask pass (gate fusion,
// qba_k_sv_xmask); each thread moves 16 B (a double2) per access whenever
// the touched bits allow it, so a pass is bound by HBM at 16 B of traffic
// per amplitude it moves (8 B read + 8 B written).
#include "qba_compact.h"

static constexpr double kInvSqrt2 = 0.70710678118654752440;

__device__ __forceinline__ uint64_t qba_ins0(uint64_t i, int b) {  // insert a 0 bit at position b
  const uint64_t lo = i & ((1ull << b) - 1ull);
  return ((i >> b) << (b + 1)) | lo;
}

__global__ void qba_k_sv_init(double2 *__restrict__ sv, uint64_t n2) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n2;
       i += (uint64_t)gridDim.x * blockDim.x)
    sv[i] = make_double2(i == 0 ? 1.0 : 0.0, 0.0);
}

// Hadamard on the qubit at bit position b (nq-1-target).
// b >= 1: thread t handles the two adjacent pairs rooted at ins0(2t, b).
__global__ void qba_k_sv_h(double *__restrict__ sv, int b, uint64_t nthreads) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads;
       t += (uint64_t)gridDim.x * blockDim.x) {
    if (b == 0) {
      double2 *p = reinterpret_cast<double2 *>(sv) + t;
      const double2 a = *p;
      *p = make_double2((a.x + a.y) * kInvSqrt2, (a.x - a.y) * kInvSqrt2);
    } else {
      const uint64_t i0 = qba_ins0(2 * t, b);
      double2 *p0 = reinterpret_cast<double2 *>(sv + i0);
      double2 *p1 = reinterpret_cast<double2 *>(sv + i0 + (1ull << b));
      const double2 a = *p0, c = *p1;
      *p0 = make_double2((a.x + c.x) * kInvSqrt2, (a.y + c.y) * kInvSqrt2);
      *p1 = make_double2((a.x - c.x) * kInvSqrt2, (a.y - c.y) * kInvSqrt2);
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
      const double2 a = *p0;
      if (M & 1ull) {
        double2 *p1 = reinterpret_cast<double2 *>(sv + (j - 1));
        const double2 c = *p1;
        *p0 = make_double2(c.y, c.x);
        *p1 = make_double2(a.y, a.x);
      } else {
        double2 *p1 = reinterpret_cast<double2 *>(sv + j);
        *p0 = *p1;
        *p1 = a;
      }
    } else {
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

extern "C" int qba_sv_init(qba_ctx *ctx, double *sv, int nq, qba_stream stream) {
  if (!ctx || !sv || nq < 1 || nq > 40) return qba_fail(QBA_EINVAL, "qba_sv_init: bad arguments");
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  const uint64_t n2 = 1ull << (nq - 1);
  hipLaunchKernelGGL(qba_k_sv_init, dim3(sv_grid(n2)), dim3(256), 0, (hipStream_t)stream,
                     reinterpret_cast<double2 *>(sv), n2);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

extern "C" int qba_sv_apply(qba_ctx *ctx, double *sv, int nq, const int32_t *gates, int ngates,
                            qba_stream stream) {
  if (!ctx || !sv || nq < 1 || nq > 40 || ngates < 0 || (ngates && !gates))
    return qba_fail(QBA_EINVAL, "qba_sv_apply: bad arguments");
  for (int g = 0; g < ngates; ++g) {  // validate everything before launching anything
    const int32_t k = gates[3 * g], t = gates[3 * g + 1], c = gates[3 * g + 2];
    if ((k != QBA_GATE_H && k != QBA_GATE_X) || t < 0 || t >= nq || c >= nq || c == t ||
        (c < -1) || (k == QBA_GATE_H && c >= 0))
      return qba_fail(QBA_EINVAL, "qba_sv_apply: gate " + std::to_string(g) + " is invalid");
  }
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  hipStream_t s = (hipStream_t)stream;
  // runs of X gates (ctl -1) or of CX gates sharing a control fold into one
  // XOR-mask pass; H gates are one butterfly pass each
  int run_ctl = -2;  // -2: no open run
  uint64_t run_mask = 0;
  auto flush = [&]() -> int {
    if (run_ctl != -2 && run_mask) {
      const int bc = run_ctl < 0 ? -1 : nq - 1 - run_ctl;
      const int brep = 63 - __builtin_clzll(run_mask);
      const int vec = (brep != 0 && bc != 0 && nq >= (bc >= 0 ? 3 : 2)) ? 1 : 0;
      const uint64_t npairs = (1ull << (nq - 1)) >> (bc >= 0 ? 1 : 0);
      const uint64_t nthr = npairs / (vec ? 2 : 1);
      hipLaunchKernelGGL(qba_k_sv_xmask, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, bc, brep, run_mask, nthr,
                         vec);
      QBA_HIP(hipGetLastError());
    }
    run_ctl = -2;
    run_mask = 0;
    return QBA_OK;
  };
  for (int g = 0; g < ngates; ++g) {
    const int32_t k = gates[3 * g], t = gates[3 * g + 1], c = gates[3 * g + 2];
    const int bt = nq - 1 - t;
    if (k == QBA_GATE_X) {
      const int ctl = c < 0 ? -1 : c;
      if (ctl != run_ctl) {
        if (int e = flush()) return e;
        run_ctl = ctl;
      }
      run_mask ^= 1ull << bt;
      continue;
    }
    if (int e = flush()) return e;
    const uint64_t nthr = bt == 0 ? (1ull << (nq - 1)) : (1ull << (nq - 1)) / 2;
    hipLaunchKernelGGL(qba_k_sv_h, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, bt, nthr);
    QBA_HIP(hipGetLastError());
  }
  return flush();
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
