// qba_plan.cpp -- host-only planning of a resource compile (see qba_plan.h).
#include "qba_plan.h"

#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <numeric>
#include <string>

namespace {
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

// What the fused pair-bin counter relies on (qba_lists_kern.h, qba_count_pb):
// every Q entry the closed sampler draws holds n+1 DISTINCT values r ^ pi(g).
// That holds when each stage-A row's bytes 0..n are a permutation of 0..n and
// each B / C selector permutes the window while fixing its bytes past n (the
// zero padding).  Checked once per program build; a violation is an error.
static bool check_perm_tables(int n, const std::vector<uint32_t> &w, uint32_t ra, uint32_t rb, uint32_t rc,
                              int offB, int offC) {
  const int base = n >= 8 ? 4 : 0;
  if (w.size() != 4 * (size_t)ra + 2 * (size_t)rb + rc || offB != 4 * (int)ra || offC != offB + 2 * (int)rb)
    return false;  // A [ra][4], B [rb][2], C [rc]: the layout the kernels index
  auto byte = [&](size_t word, int b) { return (int)((w[word] >> (8 * b)) & 0xffu); };
  for (uint32_t i = 0; i < ra; ++i) {
    uint32_t seen = 0;
    for (int b = 0; b <= n; ++b) {
      const int v = byte(4 * (size_t)i + b / 4, b % 4);
      if (v > n || (seen >> v & 1u)) return false;
      seen |= 1u << v;
    }
  }
  // a selector over window bytes [lo, hi]: a permutation of them fixing every byte past n
  auto perm_ok = [&](const int *sel, int lo, int hi) {
    uint32_t seen = 0;
    for (int b = lo; b <= hi; ++b) {
      const int v = sel[b - lo];
      if (v < lo || v > hi || (seen >> v & 1u)) return false;
      if (base + b > n && v != b) return false;
      seen |= 1u << v;
    }
    return true;
  };
  for (uint32_t i = 0; i < rb; ++i) {
    int sel[8];
    for (int b = 0; b < 8; ++b) sel[b] = byte((size_t)offB + 2 * i + b / 4, b % 4);
    if (!perm_ok(sel, 0, 7)) return false;
  }
  for (uint32_t i = 0; i < rc && rc > 1; ++i) {
    int sel[4];
    for (int b = 0; b < 4; ++b) sel[b] = byte((size_t)offC + i, b);
    if (!perm_ok(sel, 4, 7)) return false;
  }
  return true;
}

int qba_plan_gates(int n, int kind, const int32_t *gates, int ngates, const int32_t *perm,
                   std::vector<int32_t> &kept) {
  const int nq = qba_nq(n), N = (n + 1) * nq;
  std::vector<int32_t> g(gates, gates + 3 * ngates);
  for (int i = 0; i < ngates; ++i) {
    const int k = g[3 * i], t = g[3 * i + 1], c = g[3 * i + 2];
    if ((k != QBA_GATE_H && k != QBA_GATE_X) || t < 0 || t >= N || c >= N || c == t || c < -1 ||
        (k == QBA_GATE_H && c >= 0))
      return qba_fail(QBA_EINVAL, "qba_resource_compile: gate " + std::to_string(i) + " is invalid");
  }
  if (kind != QBA_KIND_Q) {
    kept.swap(g);
    return QBA_OK;
  }
  if (!perm) return qba_fail(QBA_EINVAL, "qba_resource_compile: the Q circuit needs its permutation");
  std::vector<int> seen(n + 1, 0);
  for (int gg = 1; gg <= n; ++gg) {
    if (perm[gg - 1] < 1 || perm[gg - 1] > n || seen[perm[gg - 1]]++)
      return qba_fail(QBA_EINVAL, "qba_resource_compile: perm is not a permutation of 1..n");
  }
  uint64_t mask = 0;
  kept.clear();
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
  return QBA_OK;
}

std::vector<std::vector<int>> qba_plan_registers(int N, const std::vector<int32_t> &g) {
  std::vector<int> par(N);
  std::iota(par.begin(), par.end(), 0);
  for (size_t i = 0; i + 2 < g.size(); i += 3)
    if (g[i + 2] >= 0) par[find(par, g[i + 1])] = find(par, g[i + 2]);
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
  return regs;
}

int qba_plan_program(int n, const std::vector<HostFactor> &facs, QbaHostProgram &hp) {
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
  hp = QbaHostProgram{};
  QbaProgram &P = hp.p;
  P.nfac = (int)merged.size();
  int word = 0, shift = 0, rc;
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
  return QBA_OK;
}

int qba_plan_image(int n, const QbaHostProgram &a, const QbaHostProgram &b, std::vector<char> &img) {
  const int nq = qba_nq(n);
  const int T = a.p.table_len + b.p.table_len;
  if (T > QBA_MAX_TABLE) return qba_fail(QBA_EUNSUPPORTED, "alias tables exceed the LDS budget");
  const bool closed = n <= QBA_CLOSED_MAX_N && notq_closed(a, n) && q_closed(b, n);
  std::vector<uint32_t> pw;
  uint32_t ra = 1, rb = 1, rc = 1;
  int offB = 0, offC = 0;
  if (closed) {
    build_perm_tables(n, pw, ra, rb, rc, offB, offC);
    if (!check_perm_tables(n, pw, ra, rb, rc, offB, offC))
      return qba_fail(QBA_EINVAL, "closed-form stage tables are not permutations (internal error)");
  }
  if (pw.size() > QBA_PERM_MAX_WORDS) return qba_fail(QBA_EINVAL, "permutation tables too large");
  // stage tables 16-B aligned and padded to whole 16-B words: the list kernels
  // stage them into LDS with 16-B loads
  const size_t perm_off = QBA_PERM_OFF;
  const size_t tab_off = perm_off + sizeof(uint32_t) * ((pw.size() + 3) & ~(size_t)3);
  img.assign(tab_off + 3 * sizeof(uint64_t) * (size_t)T, 0);
  QbaProgramSet *ps = reinterpret_cast<QbaProgramSet *>(img.data());
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
  ps->perm_off = (int32_t)perm_off;
  ps->tab_off = (int32_t)tab_off;
  if (closed) {
    ps->nfact = (uint32_t)factorial(n);
    ps->t32 = (uint32_t)((1ull << 32) % ps->nfact);
    ps->ra = ra;
    ps->rb = rb;
    ps->rc = rc;
    ps->perm_words = (int32_t)pw.size();
    if (!pw.empty()) memcpy(img.data() + perm_off, pw.data(), sizeof(uint32_t) * pw.size());
  }
  uint64_t *tab = reinterpret_cast<uint64_t *>(img.data() + tab_off);
  std::copy(a.pat.begin(), a.pat.end(), tab);
  std::copy(b.pat.begin(), b.pat.end(), tab + a.pat.size());
  std::copy(a.apat.begin(), a.apat.end(), tab + T);
  std::copy(b.apat.begin(), b.apat.end(), tab + T + a.apat.size());
  std::copy(a.thr.begin(), a.thr.end(), tab + 2 * T);
  std::copy(b.thr.begin(), b.thr.end(), tab + 2 * T + a.thr.size());
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
