/*
 * sanitize_main.c -- drives the C twin (sampler_ref.c) under AddressSanitizer
 * and UBSan: `make -C oracle sanitize` then oracle/lib/sanitize_check
 * (tests/test_sanitizers.py).  TEST INFRASTRUCTURE ONLY.
 *
 * Exercises every exported entry point on small inputs: Philox, the
 * closed-form and the program-driven samplers (a hand-built uniform program
 * and a non-uniform one), counts over materialised lists (incl. values >= w),
 * the streaming and the batched counters, and checks they agree.
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

void oracle_philox(const uint32_t *ctr, int64_t n, uint64_t key, uint32_t *out);
void oracle_sample(int n, uint64_t seed, uint64_t first, uint64_t count, int closed, int nfac0,
                   const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0, const uint64_t *thr0,
                   int nfac1, const int32_t *desc1, const uint64_t *pat1, const uint64_t *apat1,
                   const uint64_t *thr1, uint8_t *lists, uint64_t ld);
int64_t oracle_counts(int n, const uint8_t *lists, uint64_t count, uint64_t ld, int64_t *H, int64_t *Cc, int64_t *P);
int64_t oracle_stream_counts(int n, uint64_t seed, uint64_t first, uint64_t count, int closed, int nfac0,
                             const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                             const uint64_t *thr0, int nfac1, const int32_t *desc1, const uint64_t *pat1,
                             const uint64_t *apat1, const uint64_t *thr1, int64_t *H, int64_t *Cc, int64_t *P);
void oracle_batched_counts(int n, uint64_t seed_base, int64_t n_inst, uint64_t count, int closed, int nfac0,
                           const int32_t *desc0, const uint64_t *pat0, const uint64_t *apat0,
                           const uint64_t *thr0, int nfac1, const int32_t *desc1, const uint64_t *pat1,
                           const uint64_t *apat1, const uint64_t *thr1, int64_t *H, int64_t *Cc, int64_t *P);

static int fails = 0;
#define CHECK(c, msg)                                     \
  do {                                                    \
    if (!(c)) {                                           \
      ++fails;                                            \
      fprintf(stderr, "FAIL line %d: %s\n", __LINE__, msg); \
    }                                                     \
  } while (0)

static int nq_of(int n) {
  int q = 0;
  while ((1 << q) < n + 1) ++q;
  return q;
}

int main(void) {
  /* Philox KAT (Random123): counter 0, key 0 */
  const uint32_t ctr[4] = {0, 0, 0, 0};
  uint32_t out[4];
  oracle_philox(ctr, 1, 0, out);
  CHECK(out[0] == 0x6627E8D5u && out[3] == 0x9B00DBD8u, "philox KAT");

  /* n = 3 program: not-Q = one factor of 6 bits (L0 = L1: patterns built
     from 64 columns), Q = one GHZ factor; a second, non-uniform Q program */
  const int n = 3, nq = nq_of(n), N = (n + 1) * nq, W = 1 << nq;
  int32_t d0[6] = {6, 1, 0, 0, 8, -1}, d1[6] = {2, 1, 0, 0, 1, -1}, d2[6] = {2, 0, 0, 0, 1, 1};
  uint64_t pat0[64], pat1[4], apat1[4], thr1[4];
  for (int c = 0; c < 64; ++c) { /* fields 1..3 = the three 2-bit digits of c, field 0 = field 1 */
    const uint64_t f1 = c & 3, f2 = (c >> 2) & 3, f3 = (c >> 4) & 3;
    pat0[c] = f1 << (N - nq) | f1 << (N - 2 * nq) | f2 << (N - 3 * nq) | f3 << (N - 4 * nq);
  }
  for (int r = 0; r < W; ++r) {
    pat1[r] = 0;
    for (int g = 0; g <= n; ++g) pat1[r] |= (uint64_t)r << (N - (g + 1) * nq);
    apat1[r] = pat1[(r + 1) % W];
    thr1[r] = (uint64_t)(0.75 * 4294967296.0);
  }
  const uint64_t count = 20011;
  const uint64_t ld = count + 5;
  uint8_t *lists = calloc((size_t)(n + 1) * ld, 1);
  int64_t H[16 * 16 * 16], C[16 * 16 * 16], P[16], H2[16 * 16 * 16], C2[16 * 16 * 16], P2[16];
  for (int closed = 0; closed <= 1; ++closed) {
    for (int nonuni = 0; nonuni <= 1; ++nonuni) {
      const int32_t *dq = nonuni ? d2 : d1;
      oracle_sample(n, 42, 7, count, closed, 1, d0, pat0, pat0, NULL, 1, dq, pat1, apat1, thr1, lists, ld);
      const int64_t bad = oracle_counts(n, lists, count, ld, H, C, P);
      CHECK(bad == 0, "no invalid values in sampled lists");
      const int64_t bad2 = oracle_stream_counts(n, 42, 7, count, closed, 1, d0, pat0, pat0, NULL, 1, dq, pat1, apat1,
                                                thr1, H2, C2, P2);
      CHECK(bad2 == 0 && !memcmp(H, H2, sizeof(int64_t) * W * (n + 1) * W) &&
                !memcmp(C, C2, sizeof(int64_t) * W * (n + 1) * (n + 1)) && !memcmp(P, P2, sizeof(int64_t) * W),
            "stream counts == counts of the lists");
    }
  }
  /* values >= w are reported, not counted */
  for (uint64_t k = 0; k < count; ++k)
    if (lists[k] != lists[ld + k]) {
      lists[2 * ld + k] = 200;
      break;
    }
  CHECK(oracle_counts(n, lists, count, ld, H, C, P) == 1, "one invalid entry");
  /* batched instances, closed form, n = 7 */
  const int n7 = 7, w7 = 8;
  int64_t *Hb = calloc((size_t)3 * w7 * (n7 + 1) * w7, 8), *Cb = calloc((size_t)3 * w7 * (n7 + 1) * (n7 + 1), 8),
          *Pb = calloc((size_t)3 * w7, 8);
  oracle_batched_counts(n7, 100, 3, 5003, 1, 0, NULL, NULL, NULL, NULL, 0, NULL, NULL, NULL, NULL, Hb, Cb, Pb);
  int64_t tot = 0;
  for (int i = 0; i < 3 * w7; ++i) tot += Pb[i];
  CHECK(tot > 3 * 5003 / 3 && tot < 3 * 5003 * 2 / 3, "batched Q fraction ~ 1/2");
  free(Hb);
  free(Cb);
  free(Pb);
  free(lists);
  if (fails) return 1;
  printf("sanitize_check: all C-twin checks passed (ASan/UBSan build)\n");
  return 0;
}
