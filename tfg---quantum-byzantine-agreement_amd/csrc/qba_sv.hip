// qba_sv.hip -- dense real-fp64 statevector kernels for the resource state
// (tfg.py:15-65).  H, X and controlled-X keep amplitudes real, so a state of
// q qubits is 2^q doubles (8 B each; 2^35 = 275 GB is the largest that fits
// one MI355X).  Qubit 0 is the most significant bit of the basis index.
//
// Every gate is one streaming pass over the state: each thread moves 16 B
// (a double2) per access whenever the touched bits allow it, so a pass is
// bound by HBM at 16 B of traffic per amplitude (8 B read + 8 B written).
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

// kind: 0 = H, 1 = X.  b = bit position of the target (nq-1-target).
// b >= 1: thread t handles the two adjacent pairs rooted at ins0(2t, b).
template <int KIND>
__global__ void qba_k_sv_1q(double *__restrict__ sv, int b, uint64_t nthreads) {
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads;
       t += (uint64_t)gridDim.x * blockDim.x) {
    if (b == 0) {
      double2 *p = reinterpret_cast<double2 *>(sv) + t;
      const double2 a = *p;
      *p = KIND == 0 ? make_double2((a.x + a.y) * kInvSqrt2, (a.x - a.y) * kInvSqrt2)
                     : make_double2(a.y, a.x);
    } else {
      const uint64_t i0 = qba_ins0(2 * t, b);
      double2 *p0 = reinterpret_cast<double2 *>(sv + i0);
      double2 *p1 = reinterpret_cast<double2 *>(sv + i0 + (1ull << b));
      const double2 a = *p0, c = *p1;
      if (KIND == 0) {
        *p0 = make_double2((a.x + c.x) * kInvSqrt2, (a.y + c.y) * kInvSqrt2);
        *p1 = make_double2((a.x - c.x) * kInvSqrt2, (a.y - c.y) * kInvSqrt2);
      } else {
        *p0 = c;
        *p1 = a;
      }
    }
  }
}

// controlled X: bc = control bit position, bt = target bit position.
// Threads enumerate indices with both bits clear; when neither bit is 0 a
// thread handles two adjacent indices with double2 accesses.
__global__ void qba_k_sv_cx(double *__restrict__ sv, int bc, int bt, uint64_t nthreads, int vec) {
  const int blo = bc < bt ? bc : bt, bhi = bc < bt ? bt : bc;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nthreads;
       t += (uint64_t)gridDim.x * blockDim.x) {
    if (vec) {
      const uint64_t i = qba_ins0(qba_ins0(2 * t, blo), bhi) | (1ull << bc);
      double2 *p0 = reinterpret_cast<double2 *>(sv + i);
      double2 *p1 = reinterpret_cast<double2 *>(sv + (i | (1ull << bt)));
      const double2 a = *p0;
      *p0 = *p1;
      *p1 = a;
    } else {
      const uint64_t i = qba_ins0(qba_ins0(t, blo), bhi) | (1ull << bc);
      const uint64_t j = i | (1ull << bt);
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
  for (int g = 0; g < ngates; ++g) {
    const int32_t k = gates[3 * g], t = gates[3 * g + 1], c = gates[3 * g + 2];
    const int bt = nq - 1 - t;
    if (c < 0) {
      const uint64_t nthr = bt == 0 ? (1ull << (nq - 1)) : (1ull << (nq - 1)) / 2;
      if (nq == 1 && bt == 0) {
        // a single pair handled by one thread
      }
      if (k == QBA_GATE_H)
        hipLaunchKernelGGL(qba_k_sv_1q<0>, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, bt, nthr);
      else
        hipLaunchKernelGGL(qba_k_sv_1q<1>, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, bt, nthr);
    } else {
      const int bc = nq - 1 - c;
      const int vec = (bt >= 1 && bc >= 1 && nq >= 3) ? 1 : 0;
      const uint64_t nthr = (1ull << (nq - 2)) / (vec ? 2 : 1);
      hipLaunchKernelGGL(qba_k_sv_cx, dim3(sv_grid(nthr)), dim3(256), 0, s, sv, bc, bt, nthr, vec);
    }
    QBA_HIP(hipGetLastError());
  }
  return QBA_OK;
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
