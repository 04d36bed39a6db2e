// qba_resource.hip -- compile a reference circuit into the sampler's program.
//
// notQCorrelated (tfg.py:15-22) and qCorrelated (tfg.py:25-40) build gate
// lists over N = (n+1)*nQ qubits.  N = 48 at n = 11, far beyond a dense
// state, but both circuits factor into small entangled registers (Bell pairs
// and |+> qubits; nQ GHZ registers of n+1 qubits).  Compilation:
//   1. (Q only) the permutation's X gates act on qubits that are afterwards
//      only CX targets, so they commute to the end: a classical XOR mask.
//      They are removed and checked against the permutation layout the
//      sampler draws afresh for every entry (field g = pi(g), tfg.py:33-37).
//   2. union-find over the 2-qubit gates gives the registers;
//   3. each register is simulated on the DEVICE (qba_sv_*), its support
//      compacted and mapped back to outcome bits (bit N-1-q = qubit q);
//   4. registers are merged while the product support stays <= 256 and each
//      merged factor gets a Vose alias table (uniform ones need no u draw);
//   5. the per-entry random-word schedule is fixed (see qba_internal.h).
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <vector>

#include "qba_plan.h"

static int simulate_register(qba_ctx *ctx, const std::vector<int> &qubits,
                             const std::vector<int32_t> &gates, int N, HostFactor &out) {
  const int q = (int)qubits.size();
  if (q > 30) return qba_fail(QBA_EUNSUPPORTED, "resource register wider than 30 qubits");
  std::vector<int> local(N, -1);
  for (int i = 0; i < q; ++i) local[qubits[i]] = i;
  std::vector<int32_t> g;
  for (size_t i = 0; i < gates.size(); i += 3) {
    const int t = gates[i + 1], c = gates[i + 2];
    if (local[t] < 0) continue;
    g.push_back(gates[i]);
    g.push_back(local[t]);
    g.push_back(c < 0 ? -1 : local[c]);
  }
  double *sv = nullptr;
  const size_t bytes = sizeof(double) << q;
  if (hipMalloc(&sv, bytes < 16 ? 16 : bytes) != hipSuccess)
    return qba_fail(QBA_ENOMEM, "resource register statevector allocation failed");
  struct Free {
    double *p;
    ~Free() { (void)hipFree(p); }
  } guard{sv};
  int rc;
  if (q == 0) return qba_fail(QBA_EINVAL, "empty register");
  if ((rc = qba_sv_prepare(ctx, sv, q, g.data(), (int)g.size() / 3, nullptr))) return rc;
  const int64_t cap = 1 << 16;
  int64_t *idx_d = nullptr;
  double *prob_d = nullptr;
  if (hipMalloc(&idx_d, cap * sizeof(int64_t)) != hipSuccess) return qba_fail(QBA_ENOMEM, "support buffer");
  struct Free2 {
    void *a;
    ~Free2() { (void)hipFree(a); }
  } g2{idx_d};
  if (hipMalloc(&prob_d, cap * sizeof(double)) != hipSuccess) return qba_fail(QBA_ENOMEM, "support buffer");
  struct Free3 {
    void *a;
    ~Free3() { (void)hipFree(a); }
  } g3{prob_d};
  int64_t cnt = 0;
  if ((rc = qba_sv_support(ctx, sv, q, 1e-24, idx_d, prob_d, cap, &cnt, nullptr))) return rc;
  if (cnt > 256 || cnt < 1)
    return qba_fail(QBA_EUNSUPPORTED, "register support of " + std::to_string(cnt) +
                                          " outcomes does not fit one alias table (<= 256)");
  std::vector<int64_t> idx(cnt);
  std::vector<double> prob(cnt);
  QBA_HIP(hipMemcpy(idx.data(), idx_d, cnt * sizeof(int64_t), hipMemcpyDeviceToHost));
  QBA_HIP(hipMemcpy(prob.data(), prob_d, cnt * sizeof(double), hipMemcpyDeviceToHost));
  out.pat.resize(cnt);
  out.prob = prob;
  for (int64_t s = 0; s < cnt; ++s) {
    uint64_t pattern = 0;
    for (int i = 0; i < q; ++i)
      if ((idx[s] >> (q - 1 - i)) & 1) pattern |= 1ull << (N - 1 - qubits[i]);
    out.pat[s] = pattern;
  }
  return QBA_OK;
}

extern "C" int qba_resource_compile(qba_ctx *ctx, int n, int kind, const int32_t *gates, int ngates,
                                    const int32_t *perm) {
  if (!ctx || n < 1 || n > QBA_MAX_PARTIES || (kind != QBA_KIND_NOTQ && kind != QBA_KIND_Q) ||
      ngates < 0 || (ngates && !gates))
    return qba_fail(QBA_EINVAL, "qba_resource_compile: bad arguments");
  const int N = (n + 1) * qba_nq(n);
  // 1. validation and (Q) the classical permutation mask
  std::vector<int32_t> g;
  int rc = qba_plan_gates(n, kind, gates, ngates, perm, g);
  if (rc) return rc;
  // 2. registers
  const std::vector<std::vector<int>> regs = qba_plan_registers(N, g);
  if ((rc = qba_set_device(ctx))) return rc;
  // 3. simulate each register on the device
  std::vector<HostFactor> facs(regs.size());
  for (size_t r = 0; r < regs.size(); ++r)
    if ((rc = simulate_register(ctx, regs[r], g, N, facs[r]))) return rc;
  // 4. merge and alias tables
  QbaHostProgram hp;
  if ((rc = qba_plan_program(n, facs, hp))) return rc;
  ctx->hprog[n][kind] = hp;
  ctx->compiled[n][kind] = true;
  // 5. device image once both kinds exist
  if (ctx->compiled[n][0] && ctx->compiled[n][1]) {
    std::vector<char> img;
    if ((rc = qba_plan_image(n, ctx->hprog[n][0], ctx->hprog[n][1], img))) return rc;
    const size_t bytes = img.size();
    char *host = (char *)malloc(bytes);
    if (!host) return qba_fail(QBA_ENOMEM, "host image");
    memcpy(host, img.data(), bytes);
    void *dev = nullptr;
    if (hipMalloc(&dev, bytes) != hipSuccess) {
      free(host);
      return qba_fail(QBA_ENOMEM, "program image");
    }
    if (hipMemcpy(dev, host, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      free(host);
      (void)hipFree(dev);
      return qba_fail(QBA_EHIP, "program upload");
    }
    if (ctx->prog_dev[n]) {
      (void)hipDeviceSynchronize();
      (void)hipFree(ctx->prog_dev[n]);
    }
    free(ctx->prog_host[n]);
    ctx->prog_dev[n] = dev;
    ctx->prog_host[n] = host;
    ctx->prog_bytes[n] = bytes;
  }
  return QBA_OK;
}

extern "C" int qba_program_export(qba_ctx *ctx, int n, int kind, int32_t *n_factors, int32_t *desc,
                                  uint64_t *pat, uint64_t *apat, uint64_t *thr, int32_t cap,
                                  int32_t *table_len) {
  if (!ctx || n < 1 || n > QBA_MAX_PARTIES || (kind != 0 && kind != 1) || !n_factors || !desc ||
      !table_len)
    return qba_fail(QBA_EINVAL, "qba_program_export: bad arguments");
  if (!ctx->compiled[n][kind]) return qba_fail(QBA_ESTATE, "qba_program_export: not compiled");
  const QbaHostProgram &hp = ctx->hprog[n][kind];
  *n_factors = hp.p.nfac;
  *table_len = hp.p.table_len;
  for (int f = 0; f < hp.p.nfac; ++f) {
    const QbaFactor &F = hp.p.fac[f];
    const int32_t v[6] = {F.bits, F.uniform, F.offset, F.col_word, F.col_shift, F.u_word};
    memcpy(desc + 6 * f, v, sizeof(v));
  }
  if (cap < hp.p.table_len) return qba_fail(QBA_EINVAL, "qba_program_export: table buffer too small");
  if (pat) std::copy(hp.pat.begin(), hp.pat.end(), pat);
  if (apat) std::copy(hp.apat.begin(), hp.apat.end(), apat);
  if (thr) std::copy(hp.thr.begin(), hp.thr.end(), thr);
  return QBA_OK;
}

extern "C" int qba_program_flags(qba_ctx *ctx, int n, int32_t *flags) {
  if (!ctx || n < 1 || n > QBA_MAX_PARTIES || !flags)
    return qba_fail(QBA_EINVAL, "qba_program_flags: bad arguments");
  if (!ctx->prog_host[n]) return qba_fail(QBA_ESTATE, "qba_program_flags: not compiled");
  const QbaProgramSet *ps = reinterpret_cast<const QbaProgramSet *>(ctx->prog_host[n]);
  flags[0] = ps->canonical;
  flags[1] = ps->closed;
  flags[2] = (int32_t)ps->t32;
  flags[3] = (int32_t)ps->ra;
  flags[4] = (int32_t)ps->rb;
  flags[5] = (int32_t)ps->rc;
  return QBA_OK;
}
