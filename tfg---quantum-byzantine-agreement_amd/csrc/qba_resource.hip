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

#include "qba_internal.h"

namespace {

struct HostFactor {
  std::vector<uint64_t> pat;  // outcome patterns (size K)
  std::vector<double> prob;
};

int find(std::vector<int> &par, int a) {
  while (par[a] != a) a = par[a] = par[par[a]];
  return a;
}

}  // namespace

extern "C" int qba_alias_build(const double *prob, int32_t k, uint64_t *thr, int32_t *alias) {
  if (!prob || !thr || !alias || k < 1) return qba_fail(QBA_EINVAL, "qba_alias_build: bad arguments");
  double tot = 0;
  for (int i = 0; i < k; ++i) {
    if (!(prob[i] >= 0) || !isfinite(prob[i])) return qba_fail(QBA_EINVAL, "qba_alias_build: bad probability");
    tot += prob[i];
  }
  if (!(tot > 0)) return qba_fail(QBA_EINVAL, "qba_alias_build: probabilities sum to 0");
  // Vose (1991): scaled probabilities, small/large work lists.
  std::vector<double> q(k);
  std::vector<int> small, large;
  for (int i = 0; i < k; ++i) {
    q[i] = prob[i] / tot * k;
    (q[i] < 1.0 ? small : large).push_back(i);
  }
  std::vector<double> keep(k, 1.0);
  for (int i = 0; i < k; ++i) alias[i] = i;
  while (!small.empty() && !large.empty()) {
    const int s = small.back();
    small.pop_back();
    const int l = large.back();
    keep[s] = q[s];
    alias[s] = l;
    q[l] = (q[l] + q[s]) - 1.0;
    if (q[l] < 1.0) {
      large.pop_back();
      small.push_back(l);
    }
  }
  for (int i : large) keep[i] = 1.0;
  for (int i : small) keep[i] = 1.0;  // numerical leftovers
  for (int i = 0; i < k; ++i) {
    const double t = keep[i] * 4294967296.0;
    thr[i] = t >= 4294967296.0 ? (1ull << 32) : (uint64_t)llround(t);
  }
  return QBA_OK;
}

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
  if ((rc = qba_sv_init(ctx, sv, q, nullptr))) return rc;
  if ((rc = qba_sv_apply(ctx, sv, q, g.data(), (int)g.size() / 3, nullptr))) return rc;
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

static uint64_t factorial(int n) {
  uint64_t f = 1;
  for (int i = 2; i <= n; ++i) f *= (uint64_t)i;
  return f;
}


// ---------------------------------------------------------------------------
// Closed form.  The not-Q program is exactly "L0 = L1, L1..Ln independent
// uniform" iff (i) every factor is uniform with distinct patterns, (ii) the
// factors touch disjoint bits, (iii) in every pattern the bits of field 0 equal
// those of field 1 and (iv) the factors carry n*nQ bits in all: the choices
// then map one-to-one onto the W^n words with field0 == field1.  The Q program
// (permutation mask removed) is the GHZ register iff it is one uniform factor
// whose patterns are exactly {r in every field : r < W}.
// ---------------------------------------------------------------------------
static bool notq_closed(const QbaHostProgram &hp, int n) {
  const int nq = qba_nq(n), N = (n + 1) * nq;
  uint64_t seen_mask = 0;
  int bits = 0;
  for (int f = 0; f < hp.p.nfac; ++f) {
    const QbaFactor &F = hp.p.fac[f];
    if (!F.uniform) return false;
    const int K = 1 << F.bits;
    std::vector<uint64_t> pats(hp.pat.begin() + F.offset, hp.pat.begin() + F.offset + K);
    uint64_t m = 0;
    for (uint64_t p : pats) {
      m |= p;
      for (int j = 0; j < nq; ++j) {
        const int b0 = N - 1 - j, b1 = N - 1 - (nq + j);  // qubit j of field 0 / field 1
        if (((p >> b0) & 1) != ((p >> b1) & 1)) return false;
      }
    }
    std::sort(pats.begin(), pats.end());
    if (std::adjacent_find(pats.begin(), pats.end()) != pats.end()) return false;
    if (m & seen_mask) return false;
    seen_mask |= m;
    bits += F.bits;
  }
  return bits == n * nq;
}

static bool q_closed(const QbaHostProgram &hp, int n) {
  const int nq = qba_nq(n), N = (n + 1) * nq, W = 1 << nq;
  if (hp.p.nfac != 1 || !hp.p.fac[0].uniform || hp.p.fac[0].bits != nq) return false;
  std::vector<uint64_t> got(hp.pat.begin() + hp.p.fac[0].offset,
                            hp.pat.begin() + hp.p.fac[0].offset + W), want;
  for (int r = 0; r < W; ++r) {
    uint64_t p = 0;
    for (int g = 0; g <= n; ++g) p |= (uint64_t)r << (N - (g + 1) * nq);
    want.push_back(p);
  }
  std::sort(got.begin(), got.end());
  return got == want;
}

// Stage tables of the closed-form permutation (forward Fisher-Yates over
// positions 1..n, digit d_i in [0, n-i+1) swaps positions i and i+d_i).
//   A (n >= 8): digits of positions 1..3 -> the whole 12-byte array after
//      those swaps, 4 words per entry (bytes 0..11, word 3 unused);
//   window: the 8 bytes that hold the remaining positions (bytes 4..11 when
//      n >= 8, else bytes 0..7 with positions 1..n);
//   B: the first (up to) four window digits -> v_perm_b32 selectors {lo, hi}
//      of the window (out byte b = in byte sel[b]); C: the rest, whose swaps
//      stay inside window bytes 4..7 -> the hi selector only.
// Index of a stage = its digits in mixed radix, first digit most significant;
// the three stage indices are the mixed-radix digits (A, B, C) of the rank.
static void build_perm_tables(int n, std::vector<uint32_t> &words, uint32_t &ra, uint32_t &rb,
                              uint32_t &rc, int &offB, int &offC) {
  const bool stageA = n >= 8;
  const int base = stageA ? 4 : 0;  // first byte of the window
  std::vector<int> pos;             // window-local positions that move
  for (int p = stageA ? 4 : 1; p <= n; ++p) pos.push_back(p - base);
  const int k = (int)pos.size();
  std::vector<int> radB, radC;
  for (int i = 0; i + 1 < k; ++i) (i < 4 ? radB : radC).push_back(k - i);
  auto prod = [](const std::vector<int> &r) {
    uint32_t x = 1;
    for (int v : r) x *= (uint32_t)v;
    return x;
  };
  ra = stageA ? (uint32_t)(n * (n - 1) * (n - 2)) : 1u;
  rb = prod(radB);
  rc = prod(radC);
  words.clear();
  for (uint32_t idx = 0; idx < ra; ++idx) {
    uint8_t arr[16];
    for (int p = 0; p < 16; ++p) arr[p] = (uint8_t)(p <= n ? p : 0);
    if (stageA) {
      const int d1 = (int)(idx / ((n - 1) * (n - 2))), d2 = (int)(idx / (n - 2) % (n - 1)),
                d3 = (int)(idx % (n - 2));
      const int d[3] = {d1, d2, d3};
      for (int i = 1; i <= 3; ++i) std::swap(arr[i], arr[i + d[i - 1]]);
    }
    for (int w = 0; w < 4; ++w)
      words.push_back((uint32_t)arr[4 * w] | (uint32_t)arr[4 * w + 1] << 8 |
                      (uint32_t)arr[4 * w + 2] << 16 | (uint32_t)arr[4 * w + 3] << 24);
  }
  auto stage = [&](const std::vector<int> &rad, int first, bool hi_only) {
    const uint32_t R = prod(rad);
    for (uint32_t idx = 0; idx < R; ++idx) {
      int sel[8];
      for (int b = 0; b < 8; ++b) sel[b] = b;
      uint32_t rem = idx, div = R;
      for (size_t t = 0; t < rad.size(); ++t) {
        div /= (uint32_t)rad[t];
        const int d = (int)(rem / div);
        rem %= div;
        const int i = first + (int)t;
        std::swap(sel[pos[i]], sel[pos[i + d]]);
      }
      if (!hi_only)
        words.push_back((uint32_t)sel[0] | (uint32_t)sel[1] << 8 | (uint32_t)sel[2] << 16 |
                        (uint32_t)sel[3] << 24);
      words.push_back((uint32_t)sel[4] | (uint32_t)sel[5] << 8 | (uint32_t)sel[6] << 16 |
                      (uint32_t)sel[7] << 24);
    }
  };
  offB = (int)words.size();
  stage(radB, 0, false);
  offC = (int)words.size();
  // C's swaps all lie in window bytes 4..7 (its first position is the
  // window's fifth): its lo selector is the identity and is not stored.
  if (!radC.empty() && pos[radB.size()] < 4) {  // never: B takes the first four positions
    words.clear();
    return;
  }
  stage(radC, (int)radB.size(), true);
}

extern "C" int qba_resource_compile(qba_ctx *ctx, int n, int kind, const int32_t *gates, int ngates,
                                    const int32_t *perm) {
  if (!ctx || n < 1 || n > QBA_MAX_PARTIES || (kind != QBA_KIND_NOTQ && kind != QBA_KIND_Q) ||
      ngates < 0 || (ngates && !gates))
    return qba_fail(QBA_EINVAL, "qba_resource_compile: bad arguments");
  const int nq = qba_nq(n), N = (n + 1) * nq;
  std::vector<int32_t> g(gates, gates + 3 * ngates);
  for (int i = 0; i < ngates; ++i) {
    const int k = g[3 * i], t = g[3 * i + 1], c = g[3 * i + 2];
    if ((k != QBA_GATE_H && k != QBA_GATE_X) || t < 0 || t >= N || c >= N || c == t || c < -1 ||
        (k == QBA_GATE_H && c >= 0))
      return qba_fail(QBA_EINVAL, "qba_resource_compile: gate " + std::to_string(i) + " is invalid");
  }
  // 1. classical X mask (Q circuit)
  if (kind == QBA_KIND_Q) {
    if (!perm) return qba_fail(QBA_EINVAL, "qba_resource_compile: the Q circuit needs its permutation");
    std::vector<int> seen(n + 1, 0);
    for (int gg = 1; gg <= n; ++gg) {
      if (perm[gg - 1] < 1 || perm[gg - 1] > n || seen[perm[gg - 1]]++)
        return qba_fail(QBA_EINVAL, "qba_resource_compile: perm is not a permutation of 1..n");
    }
    uint64_t mask = 0;
    std::vector<int32_t> kept;
    for (int i = 0; i < ngates; ++i) {
      const int k = g[3 * i], t = g[3 * i + 1], c = g[3 * i + 2];
      bool classical = false;
      if (k == QBA_GATE_X && c < 0) {
        classical = true;  // every later gate touching t must be a CX with target t
        for (int j = i + 1; j < ngates && classical; ++j) {
          const int kj = g[3 * j], tj = g[3 * j + 1], cj = g[3 * j + 2];
          if (cj == t) classical = false;
          if (tj == t && !(kj == QBA_GATE_X && cj >= 0)) classical = false;
        }
      }
      if (classical) {
        mask ^= 1ull << (N - 1 - t);
      } else {
        kept.insert(kept.end(), {k, t, c});
      }
    }
    uint64_t want = 0;
    for (int gg = 1; gg <= n; ++gg) want |= (uint64_t)perm[gg - 1] << (N - (gg + 1) * nq);
    if (mask != want)
      return qba_fail(QBA_EINVAL,
                      "qba_resource_compile: the Q circuit's X gates are not the permutation mask "
                      "field g = pi(g) (tfg.py:33-37)");
    g.swap(kept);
    ngates = (int)g.size() / 3;
  }
  // 2. registers
  std::vector<int> par(N);
  std::iota(par.begin(), par.end(), 0);
  for (int i = 0; i < ngates; ++i)
    if (g[3 * i + 2] >= 0) par[find(par, g[3 * i + 1])] = find(par, g[3 * i + 2]);
  std::vector<std::vector<int>> regs;
  std::vector<int> reg_of(N, -1);
  for (int qb = 0; qb < N; ++qb) {  // ascending smallest qubit
    const int r = find(par, qb);
    if (reg_of[r] < 0) {
      reg_of[r] = (int)regs.size();
      regs.emplace_back();
    }
    regs[reg_of[r]].push_back(qb);
  }
  int rc = qba_set_device(ctx);
  if (rc) return rc;
  // 3. simulate each register on the device
  std::vector<HostFactor> facs(regs.size());
  for (size_t r = 0; r < regs.size(); ++r)
    if ((rc = simulate_register(ctx, regs[r], g, N, facs[r]))) return rc;
  // 4. merge (product support <= 256) and build the tables
  std::vector<HostFactor> merged;
  for (auto &f : facs) {
    if (!merged.empty() && merged.back().pat.size() * f.pat.size() <= 256) {
      HostFactor m;
      for (size_t a = 0; a < merged.back().pat.size(); ++a)
        for (size_t b = 0; b < f.pat.size(); ++b) {
          m.pat.push_back(merged.back().pat[a] ^ f.pat[b]);
          m.prob.push_back(merged.back().prob[a] * f.prob[b]);
        }
      merged.back() = std::move(m);
    } else {
      merged.push_back(f);
    }
  }
  if (merged.size() > QBA_MAX_FACTORS)
    return qba_fail(QBA_EUNSUPPORTED, "resource needs more than 16 alias tables");
  QbaHostProgram hp;
  QbaProgram &P = hp.p;
  P.nfac = (int)merged.size();
  int word = 0, shift = 0;
  for (size_t f = 0; f < merged.size(); ++f) {
    const int K = (int)merged[f].pat.size();
    int bits = 0;
    while ((1 << bits) < K) ++bits;
    const int Kp = 1 << bits;
    bool uniform = (K == Kp);
    for (int i = 0; i < K && uniform; ++i) uniform = fabs(merged[f].prob[i] * K - 1.0) < 1e-9;
    QbaFactor &F = P.fac[f];
    F.bits = bits;
    F.uniform = uniform ? 1 : 0;
    F.offset = (int)hp.pat.size();
    if (shift + bits > 32) {
      ++word;
      shift = 0;
    }
    F.col_word = word;
    F.col_shift = shift;
    shift += bits;
    F.u_word = -1;
    if (!uniform) {
      if (shift > 0) {
        ++word;
        shift = 0;
      }
      F.u_word = word++;
    }
    std::vector<double> pr(Kp, 0.0);
    for (int i = 0; i < K; ++i) pr[i] = merged[f].prob[i];
    std::vector<uint64_t> thr(Kp);
    std::vector<int32_t> alias(Kp);
    if ((rc = qba_alias_build(pr.data(), Kp, thr.data(), alias.data()))) return rc;
    for (int i = 0; i < Kp; ++i) {
      const uint64_t p_i = i < K ? merged[f].pat[i] : merged[f].pat[alias[i] < K ? alias[i] : 0];
      hp.pat.push_back(p_i);
      hp.apat.push_back(alias[i] < K ? merged[f].pat[alias[i]] : p_i);
      hp.thr.push_back(uniform ? (1ull << 32) : thr[i]);
    }
    if (!uniform) P.any_nonuniform = 1;
  }
  P.table_len = (int)hp.pat.size();
  const uint64_t s = factorial(n);
  P.perm_t = (0ull - s) % s;  // 2^64 mod n!
  P.valid = 1;
  ctx->hprog[n][kind] = hp;
  ctx->compiled[n][kind] = true;
  // 5. device image once both kinds exist
  if (ctx->compiled[n][0] && ctx->compiled[n][1]) {
    const QbaHostProgram &a = ctx->hprog[n][0], &b = ctx->hprog[n][1];
    const int T = a.p.table_len + b.p.table_len;
    if (T > QBA_MAX_TABLE)
      return qba_fail(QBA_EUNSUPPORTED, "alias tables exceed the LDS budget");
    const bool closed = n <= QBA_CLOSED_MAX_N && notq_closed(a, n) && q_closed(b, n);
    std::vector<uint32_t> pw;
    uint32_t ra = 1, rb = 1, rc = 1;
    int offB = 0, offC = 0;
    if (closed) build_perm_tables(n, pw, ra, rb, rc, offB, offC);
    if (pw.size() > QBA_PERM_MAX_WORDS) return qba_fail(QBA_EINVAL, "permutation tables too large");
    const size_t perm_off = sizeof(QbaProgramSet) + 3 * sizeof(uint64_t) * (size_t)T;
    const size_t bytes = perm_off + sizeof(uint32_t) * pw.size();
    char *img = (char *)calloc(1, bytes);
    if (!img) return qba_fail(QBA_ENOMEM, "host image");
    QbaProgramSet *ps = reinterpret_cast<QbaProgramSet *>(img);
    ps->prog[0] = a.p;
    ps->prog[1] = b.p;
    for (int f = 0; f < b.p.nfac; ++f) ps->prog[1].fac[f].offset += a.p.table_len;
    ps->table_total = T;
    ps->any_nonuniform = a.p.any_nonuniform | b.p.any_nonuniform;
    ps->n = n;
    ps->canonical = 1;
    {
      const int nbits = n * nq, nf = (nbits + 7) / 8;
      const QbaProgram &pa = ps->prog[0], &pb = ps->prog[1];
      if (pa.nfac != nf || pb.nfac != 1 || ps->any_nonuniform) ps->canonical = 0;
      for (int f = 0; f < pa.nfac && ps->canonical; ++f) {
        const QbaFactor &F = pa.fac[f];
        const int want_bits = f < nf - 1 ? 8 : nbits - 8 * (nf - 1);
        if (F.bits != want_bits || !F.uniform || F.offset != 256 * f || F.col_word != f / 4 ||
            F.col_shift != 8 * (f % 4))
          ps->canonical = 0;
      }
      const QbaFactor &Q = pb.fac[0];
      if (Q.bits != nq || !Q.uniform || Q.col_word != 0 || Q.col_shift != 0 ||
          Q.offset != a.p.table_len || a.p.table_len != 256 * (nf - 1) + (1 << (nbits - 8 * (nf - 1))))
        ps->canonical = 0;
    }
    ps->closed = closed ? 1 : 0;
    if (closed) {
      ps->nfact = (uint32_t)factorial(n);
      ps->t32 = (uint32_t)((1ull << 32) % ps->nfact);
      ps->ra = ra;
      ps->rb = rb;
      ps->rc = rc;
      ps->perm_off = (int32_t)perm_off;
      ps->perm_words = (int32_t)pw.size();
      (void)offB;
      (void)offC;
      memcpy(img + perm_off, pw.data(), sizeof(uint32_t) * pw.size());
    }
    uint64_t *tab = reinterpret_cast<uint64_t *>(ps + 1);
    std::copy(a.pat.begin(), a.pat.end(), tab);
    std::copy(b.pat.begin(), b.pat.end(), tab + a.pat.size());
    std::copy(a.apat.begin(), a.apat.end(), tab + T);
    std::copy(b.apat.begin(), b.apat.end(), tab + T + a.apat.size());
    std::copy(a.thr.begin(), a.thr.end(), tab + 2 * T);
    std::copy(b.thr.begin(), b.thr.end(), tab + 2 * T + a.thr.size());
    void *dev = nullptr;
    if (hipMalloc(&dev, bytes) != hipSuccess) {
      free(img);
      return qba_fail(QBA_ENOMEM, "program image");
    }
    if (hipMemcpy(dev, img, bytes, hipMemcpyHostToDevice) != hipSuccess) {
      free(img);
      (void)hipFree(dev);
      return qba_fail(QBA_EHIP, "program upload");
    }
    if (ctx->prog_dev[n]) {
      (void)hipDeviceSynchronize();
      (void)hipFree(ctx->prog_dev[n]);
    }
    free(ctx->prog_host[n]);
    ctx->prog_dev[n] = dev;
    ctx->prog_host[n] = img;
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

extern "C" int qba_perm_tables(int n, uint32_t *words, int32_t cap, int32_t *sizes) {
  if (n < 1 || n > QBA_CLOSED_MAX_N || !sizes)
    return qba_fail(QBA_EINVAL, "qba_perm_tables: n must be in [1, 11]");
  std::vector<uint32_t> pw;
  uint32_t ra, rb, rc;
  int offB, offC;
  build_perm_tables(n, pw, ra, rb, rc, offB, offC);
  sizes[0] = (int32_t)ra;
  sizes[1] = (int32_t)rb;
  sizes[2] = (int32_t)rc;
  sizes[3] = offB;
  sizes[4] = offC;
  sizes[5] = (int32_t)pw.size();
  if (words) {
    if (cap < (int32_t)pw.size()) return qba_fail(QBA_EINVAL, "qba_perm_tables: buffer too small");
    std::copy(pw.begin(), pw.end(), words);
  }
  return QBA_OK;
}
