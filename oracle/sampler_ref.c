/*
 * sampler_ref.c -- CPU twin of the engine's sampler and count-mode checker.
 *
 * TEST INFRASTRUCTURE ONLY.  Loaded by tests/ (as the bit-exact checker of
 * qba_sample / qba_check_counts) and by bench.py's cpu_baseline leg; the
 * product never links or loads it.
 *
 * What it restates:
 *   - Philox4x32-10 from its published definition (Salmon et al., SC'11;
 *     Random123 philox4x32 with 10 rounds), written independently of
 *     csrc/qba_internal.h and pinned by the Random123 known-answer vectors in
 *     tests/test_oracle_golden.py;
 *   - the entry sampling schedule documented in csrc/qba_internal.h, driven
 *     by a compiled program exported from the library (the tables
 *     themselves are checked against the reference circuits' statevectors
 *     separately);
 *   - count mode: for every position k with L0[k] != L1[k] (tfg.py:327),
 *     H[u][g][L_g[k]] += 1 and C[u][g][h] += [L_g[k] == L_h[k]], u = L1[k]
 *     (the inputs of consistent(), tfg.py:87-98, at P = {k : isQ, Lc[k]=u},
 *     tfg.py:182).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#ifdef _OPENMP
#include <omp.h>
#endif

typedef unsigned __int128 u128;

/* ---------------- Philox4x32-10 ---------------- */
static void philox4x32_10(const uint32_t in[4], const uint32_t key_in[2], uint32_t out[4]) {
  static const uint32_t M0 = 0xD2511F53u, M1 = 0xCD9E8D57u;
  static const uint32_t W0 = 0x9E3779B9u, W1 = 0xBB67AE85u;
  uint32_t x[4] = {in[0], in[1], in[2], in[3]};
  uint32_t k[2] = {key_in[0], key_in[1]};
  for (int round = 0; round < 10; ++round) {
    if (round > 0) {
      k[0] += W0;
      k[1] += W1;
    }
    uint64_t prod0 = (uint64_t)M0 * (uint64_t)x[0];
    uint64_t prod1 = (uint64_t)M1 * (uint64_t)x[2];
    uint32_t y[4];
    y[0] = (uint32_t)(prod1 >> 32) ^ x[1] ^ k[0];
    y[1] = (uint32_t)prod1;
    y[2] = (uint32_t)(prod0 >> 32) ^ x[3] ^ k[1];
    y[3] = (uint32_t)prod0;
    memcpy(x, y, sizeof x);
  }
  memcpy(out, x, sizeof x);
}

void oracle_philox(const uint32_t *ctr, int64_t n, uint64_t key, uint32_t *out) {
  const uint32_t k[2] = {(uint32_t)key, (uint32_t)(key >> 32)};
  for (int64_t i = 0; i < n; ++i) philox4x32_10(ctr + 4 * i, k, out + 4 * i);
}

/* ---------------- programs ---------------- */
typedef struct {
  int nfac;
  const int32_t *desc; /* [nfac][6]: bits, uniform, offset, col_word, col_shift, u_word */
  const uint64_t *pat, *apat, *thr;
} prog_t;

typedef struct {
  uint64_t e;
  uint32_t key[2];
  uint32_t b0[4];
  int64_t cached_block;
  uint32_t cache[4];
} entry_rng;

static void block_of(entry_rng *r, uint32_t b, uint32_t out[4]) {
  const uint32_t ctr[4] = {(uint32_t)r->e, (uint32_t)(r->e >> 32), b, 0u};
  philox4x32_10(ctr, r->key, out);
}

/* word k of the table stream for circuit `kind` (see csrc/qba_internal.h) */
static uint32_t stream_word(entry_rng *r, int kind, int k) {
  const int base = kind ? 1 : 3;
  if (k < base) return r->b0[1 + k];
  const int kk = k - base;
  const int64_t blk = 1 + kk / 4;
  if (r->cached_block != blk) {
    block_of(r, (uint32_t)blk, r->cache);
    r->cached_block = blk;
  }
  return r->cache[kk % 4];
}

static uint64_t draw_program(entry_rng *r, int kind, const prog_t *p) {
  uint64_t out = 0;
  for (int f = 0; f < p->nfac; ++f) {
    const int32_t *d = p->desc + 6 * f;
    const int bits = d[0], uniform = d[1], off = d[2], cw = d[3], cs = d[4], uw = d[5];
    const uint32_t col = (stream_word(r, kind, cw) >> cs) & (uint32_t)((1u << bits) - 1u);
    uint64_t pattern = p->pat[off + col];
    if (!uniform) {
      const uint32_t u = stream_word(r, kind, uw);
      if ((uint64_t)u >= p->thr[off + col]) pattern = p->apat[off + col];
    }
    out ^= pattern;
  }
  return out;
}

static int n_qubits(int n) {
  int q = 0;
  while ((1 << q) < n + 1) ++q;
  return q;
}

static uint64_t perm_threshold(int n) { /* 2^64 mod n! */
  u128 f = 1;
  for (int i = 2; i <= n; ++i) f *= (u128)i;
  return (uint64_t)(((u128)1 << 64) % f);
}

/* Fisher-Yates driven by the mixed-radix digits of floor(F * n! / 2^64);
 * returns 1 when Lemire's acceptance test passes. */
static int draw_perm(uint64_t F, int n, uint64_t t, int perm[]) {
  for (int g = 0; g <= n; ++g) perm[g] = g;
  for (int i = n; i >= 2; --i) {
    const u128 prod = (u128)F * (u128)i;
    const int j = 1 + (int)(uint64_t)(prod >> 64);
    F = (uint64_t)prod;
    const int tmp = perm[i];
    perm[i] = perm[j];
    perm[j] = tmp;
  }
  return F >= t;
}

static uint64_t sample_outcome(int n, uint64_t seed, uint64_t e, const prog_t *notq,
                               const prog_t *q, uint64_t t) {
  entry_rng r;
  r.e = e;
  r.key[0] = (uint32_t)seed;
  r.key[1] = (uint32_t)(seed >> 32);
  r.cached_block = -1;
  block_of(&r, 0, r.b0);
  if (!(r.b0[0] & 1u)) return draw_program(&r, 0, notq);
  const int nq = n_qubits(n), N = (n + 1) * nq;
  int perm[64];
  uint64_t F = (uint64_t)r.b0[2] | ((uint64_t)r.b0[3] << 32);
  for (uint32_t a = 1; !draw_perm(F, n, t, perm); ++a) {
    uint32_t y[4];
    block_of(&r, 0x80000000u + a, y);
    F = (uint64_t)y[0] | ((uint64_t)y[1] << 32);
  }
  uint64_t mask = 0;
  for (int g = 1; g <= n; ++g) mask |= (uint64_t)perm[g] << (N - (g + 1) * nq);
  return draw_program(&r, 1, q) ^ mask;
}

/* Closed-form schedule (csrc/qba_lists.hip, "Closed-form sampler"), used by
 * the engine for n <= 11 when both programs are proven to be tfg.py's
 * circuits' distributions.  Restated here from its definition: entry e uses
 * the 64-bit half e & 1 of the Philox block of its pair e >> 1; the rank
 * R = floor(F * n! / 2^32) is decoded directly into forward Fisher-Yates
 * digits (the engine instead splits it into three table indices). */
static int lemire_ok(uint32_t F, uint32_t nfact, uint32_t t) { return (uint32_t)(F * nfact) >= t; }

static void closed_entry(int n, uint64_t seed, uint64_t e, uint8_t vals[16]) {
  const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
  const uint64_t p = e >> 1;
  const uint32_t h = (uint32_t)(e & 1);
  const uint32_t ctr[4] = {(uint32_t)p, (uint32_t)(p >> 32), 0u, 0u};
  uint32_t x[4];
  philox4x32_10(ctr, key, x);
  const uint32_t w0 = x[2 * h], w1 = x[2 * h + 1];
  const int nq = n_qubits(n);
  const uint32_t W = 1u << nq;
  if (!(w0 & 1u)) { /* not-Q: L0 = L1, L1..Ln independent uniform */
    /* group g >= 1 takes v[g - 1]: w1's low nibbles 1..3, w1's high nibbles,
     * w0's high nibbles (w0's low nibbles hold isQ and r of a Q entry) */
    static const int w1_shift[7] = {8, 16, 24, 4, 12, 20, 28};
    static const int w0_shift[4] = {4, 12, 20, 28};
    uint32_t v[11];
    for (int i = 0; i < 7; ++i) v[i] = (w1 >> w1_shift[i]) & (W - 1);
    for (int i = 0; i < 4; ++i) v[7 + i] = (w0 >> w0_shift[i]) & (W - 1);
    vals[0] = (uint8_t)v[0];
    for (int g = 1; g <= n; ++g) vals[g] = (uint8_t)v[g - 1];
    return;
  }
  uint32_t nfact = 1;
  for (int i = 2; i <= n; ++i) nfact *= (uint32_t)i;
  const uint32_t t32 = (uint32_t)((1ull << 32) % nfact);
  const uint32_t t27 = (uint32_t)(((1ull << 27) % nfact) << 5);
  uint32_t F;
  if (lemire_ok(w1, nfact, t32)) {
    F = w1;
  } else if (lemire_ok(w0 & ~31u, nfact, t27)) {
    F = w0 & ~31u;
  } else {
    int found = 0;
    F = 0;
    for (uint32_t a = 1; !found; ++a) {
      const uint32_t c2[4] = {(uint32_t)p, (uint32_t)(p >> 32), 0x80000000u + a, h};
      uint32_t y[4];
      philox4x32_10(c2, key, y);
      for (int i = 0; i < 4 && !found; ++i)
        if (lemire_ok(y[i], nfact, t32)) {
          F = y[i];
          found = 1;
        }
    }
  }
  uint32_t R = (uint32_t)(((uint64_t)F * nfact) >> 32);
  int perm[16];
  for (int q = 0; q < 16; ++q) perm[q] = q;
  uint32_t div = nfact;
  for (int i = 1; i < n; ++i) { /* digit of position i has radix n - i + 1 */
    div /= (uint32_t)(n - i + 1);
    const int d = (int)(R / div);
    R %= div;
    const int j = i + d, tmp = perm[i];
    perm[i] = perm[j];
    perm[j] = tmp;
  }
  const uint32_t r = (w0 >> 1) & (W - 1);
  for (int g = 0; g <= n; ++g) vals[g] = (uint8_t)(r ^ (uint32_t)perm[g]);
}

static void outcome_to_column(uint64_t out, int n, uint8_t *lists, uint64_t ld, uint64_t col) {
  const int nq = n_qubits(n), N = (n + 1) * nq;
  for (int g = 0; g <= n; ++g)
    lists[(uint64_t)g * ld + col] = (uint8_t)((out >> (N - (g + 1) * nq)) & ((1u << nq) - 1u));
}

void oracle_sample(int n, uint64_t seed, uint64_t first, uint64_t count, int closed, int nfac0,
                   const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                   const uint64_t *thr0, int nfac1, const int32_t *desc1, const uint64_t *pat1,
                   const uint64_t *apat1, const uint64_t *thr1, uint8_t *lists, uint64_t ld) {
  const prog_t p0 = {nfac0, desc0, pat0, apat0, thr0}, p1 = {nfac1, desc1, pat1, apat1, thr1};
  const uint64_t t = perm_threshold(n);
  if (closed) {
#pragma omp parallel for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k) {
      uint8_t vals[16];
      closed_entry(n, seed, first + (uint64_t)k, vals);
      for (int g = 0; g <= n; ++g) lists[(uint64_t)g * ld + (uint64_t)k] = vals[g];
    }
    return;
  }
#pragma omp parallel for schedule(static)
  for (int64_t k = 0; k < (int64_t)count; ++k)
    outcome_to_column(sample_outcome(n, seed, first + (uint64_t)k, &p0, &p1, t), n, lists, ld,
                      (uint64_t)k);
}

/* ---------------- count mode ---------------- */
static void count_column(const uint8_t *lists, uint64_t ld, uint64_t k, int n, int w, int64_t *H,
                         int64_t *Cc, int64_t *bad) {
  const int G = n + 1;
  const int l0 = lists[k], l1 = lists[ld + k];
  if (l0 == l1) return;
  int l[64];
  for (int g = 0; g < G; ++g) {
    l[g] = lists[(uint64_t)g * ld + k];
    if (l[g] >= w) {
      ++*bad;
      return;
    }
  }
  const int u = l1;
  for (int g = 0; g < G; ++g) H[((int64_t)u * G + g) * w + l[g]] += 1;
  for (int g = 0; g < G; ++g)
    for (int h = g + 1; h < G; ++h)
      if (l[g] == l[h]) Cc[((int64_t)u * G + g) * G + h] += 1;
}

static void finalize(int n, int w, int64_t *H, int64_t *Cc, int64_t *P) {
  const int G = n + 1;
  for (int u = 0; u < w; ++u) {
    P[u] = H[((int64_t)u * G + 1) * w + u];
    for (int g = 0; g < G; ++g) {
      Cc[((int64_t)u * G + g) * G + g] = P[u];
      for (int h = g + 1; h < G; ++h) Cc[((int64_t)u * G + h) * G + g] = Cc[((int64_t)u * G + g) * G + h];
    }
  }
}

/* H [w][n+1][w], C [w][n+1][n+1], P [w]; returns the number of invalid Q entries */
int64_t oracle_counts(int n, const uint8_t *lists, uint64_t count, uint64_t ld, int64_t *H,
                      int64_t *Cc, int64_t *P) {
  const int w = 1 << n_qubits(n), G = n + 1;
  const size_t hb = (size_t)w * G * w, cb = (size_t)w * G * G;
  memset(H, 0, hb * sizeof(int64_t));
  memset(Cc, 0, cb * sizeof(int64_t));
  int64_t bad = 0;
#pragma omp parallel
  {
    int64_t *h = calloc(hb, sizeof(int64_t)), *c = calloc(cb, sizeof(int64_t));
    int64_t b = 0;
#pragma omp for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k) count_column(lists, ld, (uint64_t)k, n, w, h, c, &b);
#pragma omp critical
    {
      for (size_t i = 0; i < hb; ++i) H[i] += h[i];
      for (size_t i = 0; i < cb; ++i) Cc[i] += c[i];
      bad += b;
    }
    free(h);
    free(c);
  }
  finalize(n, w, H, Cc, P);
  return bad;
}

/* Fused CPU baseline: sample every entry and count it, writing the lists once
 * (the same work as one qba_sample_check step).  Returns invalid entries. */
int64_t oracle_sample_counts(int n, uint64_t seed, uint64_t first, uint64_t count, int closed, int nfac0,
                             const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                             const uint64_t *thr0, int nfac1, const int32_t *desc1,
                             const uint64_t *pat1, const uint64_t *apat1, const uint64_t *thr1,
                             uint8_t *lists, uint64_t ld, int64_t *H, int64_t *Cc, int64_t *P) {
  oracle_sample(n, seed, first, count, closed, nfac0, desc0, pat0, apat0, thr0, nfac1, desc1, pat1, apat1,
                thr1, lists, ld);
  return oracle_counts(n, lists, count, ld, H, Cc, P);
}

/* values of one entry (either schedule) into vals[0..n] */
static void entry_values(int n, uint64_t seed, uint64_t e, int closed, const prog_t *p0, const prog_t *p1,
                         uint64_t t, uint8_t vals[16]) {
  if (closed) {
    closed_entry(n, seed, e, vals);
    return;
  }
  const uint64_t out = sample_outcome(n, seed, e, p0, p1, t);
  const int nq = n_qubits(n), N = (n + 1) * nq;
  for (int g = 0; g <= n; ++g) vals[g] = (uint8_t)((out >> (N - (g + 1) * nq)) & ((1u << nq) - 1u));
}

/* count one entry from its values (same rules as count_column) */
static void count_values(const uint8_t *l, int n, int w, int64_t *H, int64_t *Cc, int64_t *bad) {
  const int G = n + 1;
  if (l[0] == l[1]) return;
  for (int g = 0; g < G; ++g)
    if (l[g] >= w) {
      ++*bad;
      return;
    }
  const int u = l[1];
  for (int g = 0; g < G; ++g) H[((int64_t)u * G + g) * w + l[g]] += 1;
  for (int g = 0; g < G; ++g)
    for (int h = g + 1; h < G; ++h)
      if (l[g] == l[h]) Cc[((int64_t)u * G + g) * G + h] += 1;
}

/* Streaming sample + count over entries [first, first+count) without storing
 * the lists (sizes far beyond host memory, e.g. sizeL = 1e9 or a 2^31 chunk
 * crossing); OpenMP with per-thread histograms.  Returns invalid entries. */
int64_t oracle_stream_counts(int n, uint64_t seed, uint64_t first, uint64_t count, int closed, int nfac0,
                             const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                             const uint64_t *thr0, int nfac1, const int32_t *desc1, const uint64_t *pat1,
                             const uint64_t *apat1, const uint64_t *thr1, int64_t *H, int64_t *Cc, int64_t *P) {
  const prog_t p0 = {nfac0, desc0, pat0, apat0, thr0}, p1 = {nfac1, desc1, pat1, apat1, thr1};
  const uint64_t t = perm_threshold(n);
  const int w = 1 << n_qubits(n), G = n + 1;
  const size_t hb = (size_t)w * G * w, cb = (size_t)w * G * G;
  memset(H, 0, hb * sizeof(int64_t));
  memset(Cc, 0, cb * sizeof(int64_t));
  int64_t bad = 0;
#pragma omp parallel
  {
    int64_t *h = calloc(hb, sizeof(int64_t)), *c = calloc(cb, sizeof(int64_t));
    int64_t b = 0;
    uint8_t vals[16];
#pragma omp for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k) {
      entry_values(n, seed, first + (uint64_t)k, closed, &p0, &p1, t, vals);
      count_values(vals, n, w, h, c, &b);
    }
#pragma omp critical
    {
      for (size_t i = 0; i < hb; ++i) H[i] += h[i];
      for (size_t i = 0; i < cb; ++i) Cc[i] += c[i];
      bad += b;
    }
    free(h);
    free(c);
  }
  finalize(n, w, H, Cc, P);
  return bad;
}

/* Batched independent instances (BASELINE configs[3]): instance i uses key
 * seed_base + i over entries [0, count); counts per instance into
 * H + i*w*G*w, Cc + i*w*G*G, P + i*w.  Parallel over instances. */
void oracle_batched_counts(int n, uint64_t seed_base, int64_t n_inst, uint64_t count, int closed, int nfac0,
                           const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                           const uint64_t *thr0, int nfac1, const int32_t *desc1, const uint64_t *pat1,
                           const uint64_t *apat1, const uint64_t *thr1, int64_t *H, int64_t *Cc, int64_t *P) {
  const prog_t p0 = {nfac0, desc0, pat0, apat0, thr0}, p1 = {nfac1, desc1, pat1, apat1, thr1};
  const uint64_t t = perm_threshold(n);
  const int w = 1 << n_qubits(n), G = n + 1;
  const size_t hb = (size_t)w * G * w, cb = (size_t)w * G * G;
#pragma omp parallel for schedule(dynamic, 1)
  for (int64_t i = 0; i < n_inst; ++i) {
    int64_t *h = H + i * (int64_t)hb, *c = Cc + i * (int64_t)cb, *pp = P + i * (int64_t)w, b = 0;
    memset(h, 0, hb * sizeof(int64_t));
    memset(c, 0, cb * sizeof(int64_t));
    uint8_t vals[16];
    for (uint64_t k = 0; k < count; ++k) {
      entry_values(n, seed_base + (uint64_t)i, k, closed, &p0, &p1, t, vals);
      count_values(vals, n, w, h, c, &b);
    }
    finalize(n, w, h, c, pp);
  }
}

/* Position-weighted row checksums of the lists of entries [first, first+count)
 * without storing them: S[2g] = sum_k L_g[k], S[2g+1] = sum_k L_g[k] * (k+1)
 * (k the column within the call; unsigned 64-bit, which never wraps below
 * 2^54 columns at w <= 16).  Layout-free: bench.py computes the same sums on
 * the device from the nibble rows it wrote. */
void oracle_stream_row_sums(int n, uint64_t seed, uint64_t first, uint64_t count, int closed, int nfac0,
                            const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                            const uint64_t *thr0, int nfac1, const int32_t *desc1, const uint64_t *pat1,
                            const uint64_t *apat1, const uint64_t *thr1, uint64_t *S) {
  const prog_t p0 = {nfac0, desc0, pat0, apat0, thr0}, p1 = {nfac1, desc1, pat1, apat1, thr1};
  const uint64_t t = perm_threshold(n);
  const int G = n + 1;
  memset(S, 0, 2 * (size_t)G * sizeof(uint64_t));
#pragma omp parallel
  {
    uint64_t s[32] = {0};
    uint8_t vals[16];
#pragma omp for schedule(static)
    for (int64_t k = 0; k < (int64_t)count; ++k) {
      entry_values(n, seed, first + (uint64_t)k, closed, &p0, &p1, t, vals);
      for (int g = 0; g < G; ++g) {
        s[2 * g] += vals[g];
        s[2 * g + 1] += (uint64_t)vals[g] * (uint64_t)(k + 1);
      }
    }
#pragma omp critical
    for (int i = 0; i < 2 * G; ++i) S[i] += s[i];
  }
}

int oracle_threads(void) {
#ifdef _OPENMP
  return omp_get_max_threads();
#else
  return 1;
#endif
}
