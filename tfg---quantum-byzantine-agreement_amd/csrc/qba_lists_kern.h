// qba_lists_kern.h -- the data-parallel hot path on gfx950 (kernels and their
// per-n launchers; instantiated by qba_lists_inst.hip):
//   * Born sampling of list entries (tfg.py:68-84 + 128-129) from the compiled
//     factored alias-table program, Philox4x32-10 keyed by the global entry;
//   * the count-mode check pass (tfg.py:87-98, 182, 189, 291-294, 327):
//     per Q-correlated entry, H[u][g][x] += 1 for every group g and
//     C[u][g][h] += 1 for every equal pair, u = L1[k];
//   * the fused sample+check kernel that writes each list byte once and
//     counts from registers.
//
// Layout: lists[g][k] uint8, row stride ld (SoA: a party's list is one row).
// A thread owns 2 x 4 consecutive entries per step (8 B per row), so every row
// store / load of a wave is 512 contiguous bytes.  Histograms are privatised per
// workgroup in LDS and flushed as u32 partials to a slab that a second
// kernel reduces into int64 (bitwise reproducible, no global atomics).
#pragma once
#include <type_traits>

#include "qba_lists.h"

// Measured shapes of the list kernels (the rejected
// alternatives and the attribution probes live in tools/exp/probes.patch)
constexpr int QBA_WIDE_QPT = 2;      // quads per thread-step of the wide kernels (one 8-B / 4-B row vector)
constexpr int QBA_PAIRWISE = 1;      // closed sampler: a quad's two pairs one after the other (fewer live VGPRs)
constexpr int QBA_DEF_PAIRWISE = 0;  // ... in the deferred (configs[1]) kernel: interleaved, more ILP at 6 waves
constexpr int QBA_DEF_WAVES = 6;     // deferred kernel: waves per SIMD it is compiled for
constexpr int QBA_GRID_QPT = 2;      // quads per thread the grid is sized for
constexpr int QBA_RED_ROWS = 32;     // slab rows per reduce workgroup

template <int NP>
struct QCfg {
  static constexpr int G = NP + 1;  // measured groups (n parties + the commander's extra)
  static constexpr int NQ = (G <= 2) ? 1 : (G <= 4) ? 2 : (G <= 8) ? 3 : 4;
  static constexpr int N = G * NQ;  // qubits of the circuit (tfg.py:44)
  static constexpr int W = 1 << NQ;  // |W| (tfg.py:318)
  static constexpr int HB = W * G * W;    // H as returned: [u][g][x]
  static constexpr int WP = W + 1;        // LDS row stride of H: +1 word spreads banks
  static constexpr int HBL = W * G * WP;  // H as counted in LDS / the slab
  static constexpr int CB = W * G * G;      // C as returned: [u][g][h]
  static constexpr int CP = G * (G - 1) / 2; // pairs g < h, as counted
  static constexpr int CBL = W * CP;
  static constexpr int STATS = 2;  // [0] Q entries with a value >= W (invalid), [1] spare
  static constexpr int NBINS = HBL + CBL + STATS;
  static constexpr int NBP = (NBINS + 3) & ~3;  // slab row stride (16-B rows)
  // counted index of the pair g < h
  __host__ __device__ static constexpr int pidx(int g, int h) { return g * (2 * G - g - 1) / 2 + (h - g - 1); }
  __host__ __device__ static constexpr int hidx(int u, int g, int x) { return (u * G + g) * WP + x; }
  // number of not-Q table bytes of the canonical program (ceil(n*nQ/8))
  static constexpr int NFB = (NP * NQ + 7) / 8;
  static constexpr int LASTB = NP * NQ - 8 * (NFB - 1);
  using Out = typename std::conditional<(N <= 32), uint32_t, uint64_t>::type;
  static constexpr Out M = (Out)(W - 1);
  __host__ __device__ static constexpr int shift(int g) { return N - (g + 1) * NQ; }
  __host__ __device__ static constexpr Out identity() {
    Out p = 0;
    for (int g = 1; g <= NP; ++g) p |= (Out)g << shift(g);
    return p;
  }
};

// ---------------------------------------------------------------------------
// random words of one entry (schedule documented in qba_internal.h)
// ---------------------------------------------------------------------------
// Words beyond block 0 (only programs with many or non-uniform factors):
// kept out of line so the common path stays small.
__device__ __attribute__((noinline)) uint32_t qba_word_ext(int kk, uint32_t elo, uint32_t ehi,
                                                           uint32_t k0, uint32_t k1) {
  const QbaU4 y = qba_philox(elo, ehi, 1u + (uint32_t)(kk >> 2), 0u, k0, k1);
  const int s = kk & 3;
  return s == 0 ? y.x : (s == 1 ? y.y : (s == 2 ? y.z : y.w));
}

// Word k of the table stream (k is wave-uniform).  Block-0 words are picked
// with uniform masks so the selection stays in registers.
__device__ __forceinline__ uint32_t qba_word(int kind, int k, const QbaU4 &x, uint32_t elo,
                                             uint32_t ehi, uint32_t k0, uint32_t k1) {
  k = __builtin_amdgcn_readfirstlane(k);
  const int base = kind ? 1 : 3;
  if (k >= base) return qba_word_ext(k - base, elo, ehi, k0, k1);
  const uint32_t m0 = k == 0 ? ~0u : 0u, m1 = k == 1 ? ~0u : 0u, m2 = k == 2 ? ~0u : 0u;
  return (x.y & m0) | (x.z & m1) | (x.w & m2);
}

template <typename Out>
__device__ __forceinline__ Out qba_draw(const QbaProgram &P, int kind, const QbaU4 &x,
                                        uint32_t elo, uint32_t ehi, uint32_t k0, uint32_t k1,
                                        const uint64_t *pat, const uint64_t *apat,
                                        const uint64_t *thr) {
  Out out = 0;
  const int nf = P.nfac;
  for (int f = 0; f < nf; ++f) {
    const QbaFactor F = P.fac[f];
    const uint32_t wv = qba_word(kind, F.col_word, x, elo, ehi, k0, k1);
    const uint32_t col = (wv >> F.col_shift) & ((1u << F.bits) - 1u);
    uint64_t p = pat[F.offset + col];
    if (!F.uniform) {
      const uint32_t u = qba_word(kind, F.u_word, x, elo, ehi, k0, k1);
      if ((uint64_t)u >= thr[F.offset + col]) p = apat[F.offset + col];
    }
    out ^= (Out)p;
  }
  return out;
}

// Uniform permutation pi of 1..n in the outcome layout (field g = pi(g)):
// mixed-radix digits of floor(F * n! / 2^64) drive Fisher-Yates; Lemire's
// test on the final fraction makes it exactly uniform.
template <int NP>
__device__ __forceinline__ bool qba_perm(uint64_t F, uint64_t t, typename QCfg<NP>::Out &mask) {
  using C = QCfg<NP>;
  using Out = typename C::Out;
  Out P = C::identity();
#pragma unroll
  for (int i = NP; i >= 2; --i) {
    const uint64_t lo = (F & 0xffffffffull) * (uint64_t)i;
    const uint64_t hi = (F >> 32) * (uint64_t)i + (lo >> 32);
    const uint32_t d = (uint32_t)(hi >> 32);
    F = (hi << 32) | (lo & 0xffffffffull);
    const int si = C::shift(i);
    const int sj = C::N - (int)(d + 2) * C::NQ;  // field j = 1 + d
    const Out a = (P >> si) & C::M;
    const Out b = (P >> sj) & C::M;
    const Out tt = a ^ b;
    P ^= (tt << si) | (tt << sj);
  }
  mask = P;
  return F >= t;
}

template <int NP>
__device__ __forceinline__ typename QCfg<NP>::Out qba_sample_entry(
    uint64_t e, uint32_t k0, uint32_t k1, const QbaProgramSet *__restrict__ ps,
    const uint64_t *pat, const uint64_t *apat, const uint64_t *thr) {
  using Out = typename QCfg<NP>::Out;
  const uint32_t elo = (uint32_t)e, ehi = (uint32_t)(e >> 32);
  const QbaU4 x = qba_philox(elo, ehi, 0u, 0u, k0, k1);
  Out out;
  if (x.x & 1u) {  // Q-correlated shot (tfg.py:69, 74)
    const uint64_t t = ps->prog[1].perm_t;
    Out mask;
    bool ok = qba_perm<NP>((uint64_t)x.z | ((uint64_t)x.w << 32), t, mask);
    for (uint32_t a = 1; !ok; ++a) {  // probability ~ n!/2^64 per entry
      const QbaU4 y = qba_philox(elo, ehi, 0x80000000u + a, 0u, k0, k1);
      ok = qba_perm<NP>((uint64_t)y.x | ((uint64_t)y.y << 32), t, mask);
    }
    out = qba_draw<Out>(ps->prog[1], 1, x, elo, ehi, k0, k1, pat, apat, thr) ^ mask;
  } else {  // not-Q-correlated shot (tfg.py:72)
    out = qba_draw<Out>(ps->prog[0], 0, x, elo, ehi, k0, k1, pat, apat, thr);
  }
  return out;
}

// Canonical programs (QbaProgramSet::canonical): every table column is a byte
// of the stream, so the factor loop is fully unrolled at compile time.
template <int NP>
__device__ __forceinline__ typename QCfg<NP>::Out qba_sample_entry_fast(
    uint64_t e, uint32_t k0, uint32_t k1, uint64_t perm_t, int qoff, const uint64_t *pat) {
  using C = QCfg<NP>;
  using Out = typename C::Out;
  const uint32_t elo = (uint32_t)e, ehi = (uint32_t)(e >> 32);
  const QbaU4 x = qba_philox(elo, ehi, 0u, 0u, k0, k1);
  Out out;
  if (x.x & 1u) {
    Out mask;
    bool ok = qba_perm<NP>((uint64_t)x.z | ((uint64_t)x.w << 32), perm_t, mask);
    for (uint32_t a = 1; !ok; ++a) {
      const QbaU4 y = qba_philox(elo, ehi, 0x80000000u + a, 0u, k0, k1);
      ok = qba_perm<NP>((uint64_t)y.x | ((uint64_t)y.y << 32), perm_t, mask);
    }
    out = (Out)pat[qoff + (x.y & (uint32_t)C::M)] ^ mask;
  } else {
    out = 0;
#pragma unroll
    for (int f = 0; f < C::NFB; ++f) {
      const uint32_t w = f < 4 ? x.y : (f < 8 ? x.z : x.w);
      const uint32_t bits = f < C::NFB - 1 ? 8 : C::LASTB;
      const uint32_t col = (w >> (8 * (f & 3))) & ((1u << bits) - 1u);
      out ^= (Out)pat[256 * f + col];
    }
  }
  return out;
}

// ---------------------------------------------------------------------------
// Closed-form sampler (QbaProgramSet::closed; n <= 11).  Entries come in
// pairs: entry e uses half h = e & 1 of block
//   x = philox(ctr = {p_lo, p_hi, 0, 0}, key = seed),  p = e >> 1,
// i.e. the 64 bits w0 = x[2h], w1 = x[2h+1].  isQ = w0 & 1.
//   not-Q: values v_0..v_10 = the nQ low bits of the nibbles at bits
//          {8,16,24, 4,12,20,28} of w1 then {4,12,20,28} of w0;
//          group g >= 1 takes v_{g-1}, group 0 takes v_0 (= group 1,
//          tfg.py:15-22).
//   Q:     r = (w0 >> 1) & (W-1).  The rank word F is w1 if
//          F * n! mod 2^32 >= 2^32 mod n!, else w0 & ~31 (bits 5..31, a
//          27-bit fraction) if F * n! mod 2^32 >= (2^27 mod n!) << 5 (Lemire on
//          27 bits), else the words of philox(ctr = {p_lo, p_hi, 0x80000000 + a,
//          h}) for a = 1, 2, ... in order (32-bit test): exactly uniform.
//          (iA, iB, iC) = the mixed-radix digits of floor(F * n! / 2^32) in
//          radices (RA, RB, RC) [F * RA = iA:F1, F1 * RB = iB:F2, F2 * RC =
//          iC:F3], pi = stage A[iA] with its window permuted by B[iB] then
//          C[iC]; group g = r ^ pi(g) (tfg.py:25-40).
// Values are produced as bytes, group g in byte g % 4 of word g / 4.
// ---------------------------------------------------------------------------
// |P_u| = sum_x H[u][0][x]; H[u][1][x] = [x == u] |P_u| (group 1's own bin is
// never counted: L1 = u by definition of the bin).
template <int NP, typename T>
__device__ __forceinline__ int64_t qba_psize(const T *bins, int u) {
  using C = QCfg<NP>;
  int64_t s = 0;
  for (int x = 0; x < C::W; ++x) s += (int64_t)bins[C::hidx(u, 0, x)];
  return s;
}
template <int NP, typename T>
__device__ __forceinline__ int64_t qba_hval(const T *bins, int i) {  // i indexes H[u][g][x]
  using C = QCfg<NP>;
  const int u = i / (C::G * C::W), g = (i / C::W) % C::G, x = i % C::W;
  if (g == 1) return x == u ? qba_psize<NP>(bins, u) : 0;
  return (int64_t)bins[C::hidx(u, g, x)];
}

template <int NP>
struct CF {
  using C = QCfg<NP>;
  static constexpr int G = NP + 1;
  static constexpr int ND = (G + 3) / 4;          // words per entry
  static constexpr int WIN = NP >= 8 ? 1 : 0;      // first word of the 8-byte window
  static constexpr int K = NP >= 8 ? NP - 3 : NP;  // window positions that move
  static constexpr uint32_t fact(int a, int b) {   // a * (a-1) * ... * b
    uint32_t x = 1;
    for (int i = a; i >= b; --i) x *= (uint32_t)i;
    return x;
  }
  static constexpr uint32_t RA = NP >= 8 ? fact(NP, NP - 2) : 1u;
  static constexpr uint32_t RB = K >= 2 ? fact(K, (K - 3 > 2 ? K - 3 : 2)) : 1u;
  static constexpr uint32_t RC = K >= 6 ? fact(K - 4, 2) : 1u;
  static constexpr uint32_t NFACT = fact(NP, 2);
  static constexpr uint32_t T32 = (uint32_t)((1ull << 32) % NFACT);
  static constexpr uint32_t T27 = (uint32_t)(((1ull << 27) % NFACT) << 5);  // 27-bit test, scaled
  static constexpr int OFFB = 4 * (int)RA;            // in words
  static constexpr int OFFC = OFFB + 2 * (int)RB;
  static constexpr int WORDS = OFFC + (int)RC;  // C keeps only its hi selector
  static constexpr uint32_t M4 = (uint32_t)(C::W - 1) * 0x01010101u;
};

__device__ __forceinline__ uint32_t qba_perm_b(uint32_t hi, uint32_t lo, uint32_t sel) {
  return __builtin_amdgcn_perm(hi, lo, sel);
}

// Lemire acceptance of a 32-bit rank word against threshold T (scaled)
template <int NP>
__device__ __forceinline__ bool qba_accept(uint32_t F, uint32_t T) {
  return F * CF<NP>::NFACT >= T;
}

// One entry from its 64 random bits (w0, w1), in two phases so that a quad's
// table reads are issued together: qba_closed_rank (not-Q words, Lemire rank;
// (p, h) identify the entry for the rare retry) then qba_closed_finish.
struct QbaClosed {
  uint32_t nqr[4];  // not-Q words before the nibble mask (word 0 already masked)
  uint32_t rank, w0;
};

template <int NP>
__device__ __forceinline__ void qba_closed_rank(uint32_t w0, uint32_t w1, uint64_t p, uint32_t h,
                                                uint32_t k0, uint32_t k1, QbaClosed &c) {
  using F = CF<NP>;
  // group g >= 1 = nibble g of (w1 low nibbles, w1 high nibbles, w0 high
  // nibbles) in byte order, group 0 = group 1: the masked words ARE the byte
  // layout, one v_perm in all (w0's low nibbles carry isQ and r); unmasked:
  // qba_closed_finish masks every not-Q word with ~qm & M4 anyway
  c.nqr[0] = qba_perm_b(w1, w1, 0x03020101u);
  c.nqr[1] = w1 >> 4;
  c.nqr[2] = w0 >> 4;
  c.nqr[3] = 0u;
  c.w0 = w0;
  // w1 is the rank word unless its Lemire test fails (P = (2^32 mod n!) /
  // 2^32, 0.56 % at n = 11): the fallback words are chosen inside the rare
  // branch, not by a select on every entry.  The branch is tested for the
  // whole wave first (some lane fails in ~30 % of the entries): the common
  // path is one compare and one scalar branch, not the divergent branch's
  // exec-mask bookkeeping on every entry (-2.5 % cycles, VALU 77.6 -> 75.3
  // per entry, profiles/r5/uniform_branch)
  uint32_t rank = w1;
  const bool bad = !qba_accept<NP>(w1, F::T32);
  if (__builtin_expect(__builtin_amdgcn_ballot_w64(bad) != 0, 0))
  if (bad) {
    rank = w0 & ~31u;
    // both tests failed (P = 6e-4 per entry at n = 11): words of further
    // Philox blocks, in order.  A not-Q entry's rank is discarded, so only
    // Q-correlated entries retry.  (Done lane by lane on the scalar unit
    // instead, the retry freed the loop of a scratch reload but cost SGPRs
    // and 2 % more cycles: profiles/r5/ab_retry.)
    if (!qba_accept<NP>(rank, F::T27) && (w0 & 1u)) {
      bool ok = false;
      for (uint32_t t = 1; !ok; ++t) {
        const QbaU4 y = qba_philox((uint32_t)p, (uint32_t)(p >> 32), 0x80000000u + t, h, k0, k1);
        const uint32_t cand[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (!ok && qba_accept<NP>(cand[i], F::T32)) {
            ok = true;
            rank = cand[i];
          }
      }
    }
  }
  // a not-Q entry discards its table words (qba_closed_finish selects its
  // nibbles): rank 0 sends its three reads to one address per table, served
  // as an LDS broadcast, so only the Q lanes' random reads meet bank conflicts
  rank &= (uint32_t)__builtin_amdgcn_sbfe((int)w0, 0, 1);
  c.rank = rank;
}

template <int NP>
__device__ __forceinline__ void qba_closed_finish(const QbaClosed &c, const uint4 &A, const uint2 &sB,
                                                  uint32_t sC, uint32_t (&D)[CF<NP>::ND]) {
  using F = CF<NP>;
  // A.w (zero in the table) is kept alive by an empty asm, so the read stays
  // one ds_read_b128 (4 LDS cycles, a ds_read_b96 takes 8) without an OR
  uint32_t q[4] = {A.x, A.y, A.z, A.w};
  asm volatile("" ::"v"(A.w));
  const uint32_t y0 = qba_perm_b(q[F::WIN + 1], q[F::WIN], sB.x);
  uint32_t y1 = qba_perm_b(q[F::WIN + 1], q[F::WIN], sB.y);
  if constexpr (F::RC > 1) y1 = qba_perm_b(y1, y0, sC);  // stage C moves window bytes 4..7 only
  q[F::WIN] = y0;
  q[F::WIN + 1] = y1;
  // r in every byte: one v_perm (byte 0 to all four) instead of a quarter-rate
  // v_mul_lo_u32 by 0x01010101
  const uint32_t R = qba_perm_b(0u, (c.w0 >> 1) & (uint32_t)(QCfg<NP>::W - 1), 0u);
  // all ones for a Q-correlated entry: one v_bfe_i32, opaque so that each
  // word's select stays one v_bitop3 (qm ? q ^ R : nq) instead of and + cmp
  // for a mask plus a v_cndmask per word
  uint32_t qm = (uint32_t)__builtin_amdgcn_sbfe((int)c.w0, 0, 1);
  asm("" : "+v"(qm));
  // not-Q words masked by ONE shared ~qm & M4, then one v_and_or per word:
  // D = (nq_raw & nqm) | (qm & (q ^ R))  (-0.2 VALU/entry, profiles/r3/ab32_microopts_and_stores.txt)
  uint32_t nqm = ~qm & F::M4;
  asm("" : "+v"(nqm));
#pragma unroll
  for (int i = 0; i < F::ND; ++i) {
    uint32_t t = qm & (q[i] ^ R);
    asm("" : "+v"(t));
    D[i] = (c.nqr[i] & nqm) | t;
  }
}

// Stage table indices of a rank and the LDS reads.
template <int NP>
__device__ __forceinline__ void qba_closed_tables(uint32_t rank, const uint32_t *__restrict__ pl,
                                                  uint4 &A, uint2 &sB, uint32_t &sC) {
  using F = CF<NP>;
  // Each digit is the high word of one v_mad_u64_u32; the empty asm makes
  // it opaque so its table offset is ONE v_lshl_add (without it the compiler
  // rebuilt digit * stride from the 64-bit product: alignbit + and + shift).
  uint32_t iA = 0, rem = rank;
  if constexpr (F::RA > 1) {
    const uint64_t pa = (uint64_t)rem * F::RA;
    iA = (uint32_t)(pa >> 32);
    rem = (uint32_t)pa;
    asm("" : "+v"(iA));
  }
  const uint64_t pb = (uint64_t)rem * F::RB;
  uint32_t iB = (uint32_t)(pb >> 32);
  asm("" : "+v"(iB));
  uint32_t iC = F::RC > 1 ? (uint32_t)(((uint64_t)(uint32_t)pb * F::RC) >> 32) : 0u;
  if constexpr (F::RC > 1) asm("" : "+v"(iC));
  A = *reinterpret_cast<const uint4 *>(pl + 4 * iA);
  sB = *reinterpret_cast<const uint2 *>(pl + F::OFFB + 2 * iB);
  sC = F::RC > 1 ? pl[F::OFFC + iC] : 0u;
}

template <int NP>
__device__ __forceinline__ void qba_closed_half(uint32_t w0, uint32_t w1, uint64_t p, uint32_t h,
                                                uint32_t k0, uint32_t k1,
                                                const uint32_t *__restrict__ pl,
                                                uint32_t (&D)[CF<NP>::ND]) {
  QbaClosed c;
  qba_closed_rank<NP>(w0, w1, p, h, k0, k1, c);
  uint4 A;
  uint2 sB;
  uint32_t sC;
  qba_closed_tables<NP>(c.rank, pl, A, sB, sC);
  qba_closed_finish<NP>(c, A, sB, sC, D);
}

// Entry e on its own (odd pair alignment, tails): the half of its pair's block.
template <int NP>
__device__ __forceinline__ void qba_closed_entry(uint64_t e, uint32_t k0, uint32_t k1,
                                                 const uint32_t *__restrict__ pl,
                                                 uint32_t (&D)[CF<NP>::ND]) {
  const uint64_t p = e >> 1;
  const uint32_t h = (uint32_t)e & 1u;
  const QbaU4 x = qba_philox((uint32_t)p, (uint32_t)(p >> 32), 0u, 0u, k0, k1);
  qba_closed_half<NP>(h ? x.z : x.x, h ? x.w : x.y, p, h, k0, k1, pl, D);
}

// Outcome word of the table samplers -> byte layout.
template <int NP>
__device__ __forceinline__ void qba_out_to_d(typename QCfg<NP>::Out o, uint32_t (&D)[CF<NP>::ND]) {
  using C = QCfg<NP>;
#pragma unroll
  for (int i = 0; i < CF<NP>::ND; ++i) D[i] = 0;
#pragma unroll
  for (int g = 0; g < C::G; ++g)
    D[g / 4] |= ((uint32_t)(o >> C::shift(g)) & (uint32_t)C::M) << (8 * (g % 4));
}

// 4x4 byte transpose: r_i byte j = input j byte i (an involution).
__device__ __forceinline__ void qba_t4(uint32_t a, uint32_t b, uint32_t c, uint32_t d, uint32_t &r0,
                                       uint32_t &r1, uint32_t &r2, uint32_t &r3) {
  const uint32_t t0 = qba_perm_b(b, a, 0x06020400u), t1 = qba_perm_b(b, a, 0x07030501u);
  const uint32_t t2 = qba_perm_b(d, c, 0x06020400u), t3 = qba_perm_b(d, c, 0x07030501u);
  r0 = qba_perm_b(t2, t0, 0x05040100u);
  r1 = qba_perm_b(t3, t1, 0x05040100u);
  r2 = qba_perm_b(t2, t0, 0x07060302u);
  r3 = qba_perm_b(t3, t1, 0x07060302u);
}

// Inline asm in this file (here and qba_add_byte below) reads and writes
// VGPRs only: no SGPR operand is written by VALU inside an asm block, so the
// VALU-writes-SGPR -> VMEM-reads-SGPR hazard the compiler cannot see through
// asm (the cause of the faulting saddr-store experiment)
// does not arise.  Keep any new asm VGPR-only.
// v_pk_lshlrev_b16: each 16-bit half of `one` shifted by the low 4 bits of
// the same half of `amt` (the upper bits of the half are ignored by the ALU).
__device__ __forceinline__ uint32_t qba_pk_onehot(uint32_t amt, uint32_t one) {
  uint32_t r;
  asm("v_pk_lshlrev_b16 %0, %1, %2" : "=v"(r) : "v"(amt), "v"(one));
  return r;
}

// lo | hi of a word's two 16-bit halves in ONE op (an SDWA v_or with the
// upper half zeroed): the union of two 16-bit one-hot sets
__device__ __forceinline__ uint32_t qba_fold16(uint32_t u) {
  uint32_t r;
  asm("v_or_b32_sdwa %0, %1, %1 dst_sel:WORD_0 dst_unused:UNUSED_PAD src0_sel:WORD_0 src1_sel:WORD_1"
      : "=v"(r) : "v"(u));
  return r;
}

typedef __attribute__((address_space(3))) uint32_t qba_lds_u32;  // LDS word (32-bit address)

// base + byte b of x in one VALU op (v_add_u32 with an SDWA byte select)
__device__ __forceinline__ uint32_t qba_add_byte(uint32_t base, uint32_t x, int b) {
  uint32_t r;
  switch (b) {
    case 0: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_0" : "=v"(r) : "v"(base), "v"(x)); break;
    case 1: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_1" : "=v"(r) : "v"(base), "v"(x)); break;
    case 2: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_2" : "=v"(r) : "v"(base), "v"(x)); break;
    default: asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:BYTE_3" : "=v"(r) : "v"(base), "v"(x)); break;
  }
  return r;
}

// value of group g (runtime g) of an entry whose byte-layout words are w0..w3
__device__ __forceinline__ uint32_t qba_byte_of(int g, uint32_t w0, uint32_t w1, uint32_t w2, uint32_t w3) {
  const int i = g >> 2;
  const uint32_t w = i == 0 ? w0 : i == 1 ? w1 : i == 2 ? w2 : w3;
  return (w >> (8 * (g & 3))) & 0xffu;
}

// ---------------------------------------------------------------------------
// count one entry (group g = byte g % 4 of D[g / 4])
//   Q-correlated iff L0 != L1 (tfg.py:327); u = L1 (tfg.py:182);
//   H[u][g][L_g] += 1 for every g; C[u][g][h] += 1 for every equal pair --
//   every counted entry is tested (its distinct-value count: the union of
//   16-bit one-hots), the pair loop runs only when that count is below n+1.
// ---------------------------------------------------------------------------
template <int NP>
__device__ __forceinline__ void qba_count_d(const uint32_t (&D)[CF<NP>::ND], uint32_t one,
                                            uint32_t *hist, bool in_range, bool known_q = false,
                                            uint32_t hoff = 0xffffffffu) {
  using C = QCfg<NP>;
  using F = CF<NP>;
  const uint32_t l0 = D[0] & 0xffu, l1 = (D[0] >> 8) & 0xffu;
  if (!known_q && l0 == l1) return;  // the Q-entry queue holds only entries with L0 != L1
  uint32_t bad = 0;
#pragma unroll
  for (int i = 0; i < F::ND; ++i) {
    uint32_t vm = 0;  // bits that must be clear: value bits >= W of the real groups
#pragma unroll
    for (int b = 0; b < 4; ++b)
      if (4 * i + b < C::G) vm |= (0xffu & ~(uint32_t)(C::W - 1)) << (8 * b);
    bad |= D[i] & vm;
  }
  if (in_range) bad = 0;  // the caller's quad-level test found no value >= W
  if (bad) {
    atomicAdd(&hist[C::HBL + C::CBL + 0], 1u);
    return;
  }
  // hoff: the histogram's LDS byte address held in a VGPR by the caller (the
  // row base is then one v_mad_u32_u24 with the stride in an SGPR).  The row
  // index is taken to nq bits (the same single v_bfe): a trusted value is
  // < W already, and whatever the bytes hold the address stays inside this
  // workgroup's histogram + queue area (x < 256 adds at most 1 KiB).  An
  // experiment build that fed unmasked words here once indexed rows up to
  // 255 * 816 B past the histogram, beyond the LDS allocation, and faulted.
  const uint32_t l1r = (D[0] >> 8) & (uint32_t)(C::W - 1);
  if (hoff == 0xffffffffu) hoff = (uint32_t)(uintptr_t)(qba_lds_u32 *)hist;
  const uint32_t hb = hoff + l1r * (uint32_t)(C::G * C::WP * 4);
#pragma unroll
  for (int i = 0; i < F::ND; ++i) {
    const uint32_t E = D[i] << 2;  // byte b = 4 * value (< 64: no carry into the next byte)
#pragma unroll
    for (int b = 0; b < 4; ++b) {
      const int g = 4 * i + b;
      if (g < C::G && g != 1) {  // H[u][1][x] = [x == u] |P_u|, derived when reduced
        const uint32_t a = qba_add_byte(hb, E, b);
        atomicAdd((uint32_t *)((qba_lds_u32 *)(uintptr_t)a + g * C::WP), 1u);
      }
    }
  }
  // Cond3 (tfg.py:96-98): distinct iff the union of the values' 16-bit
  // one-hots (two per v_pk_lshlrev_b16) has n+1 bits
  uint32_t U = 0;
#pragma unroll
  for (int i = 0; i < F::ND; ++i) {
    uint32_t mp = 0, mq = 0;
    if (4 * i + 0 < C::G) mp |= 0x0000ffffu;
    if (4 * i + 2 < C::G) mp |= 0xffff0000u;
    if (4 * i + 1 < C::G) mq |= 0x0000ffffu;
    if (4 * i + 3 < C::G) mq |= 0xffff0000u;
    U |= (qba_pk_onehot(D[i], one) & mp) | (qba_pk_onehot(D[i] >> 8, one) & mq);
  }
  if (__popc(qba_fold16(U)) != C::G) {  // some pair collides: exact slow path
    // a compact loop (values picked by selects, no private array): this
    // path is rare and unrolling it would multiply the kernel's code size
    uint32_t *c = hist + C::HBL + l1r * C::CP;
    const uint32_t w0 = D[0], w1 = F::ND > 1 ? D[F::ND > 1 ? 1 : 0] : 0u,
                   w2 = F::ND > 2 ? D[F::ND > 2 ? 2 : 0] : 0u, w3 = F::ND > 3 ? D[F::ND > 3 ? 3 : 0] : 0u;
    int pi = 0;
#pragma nounroll
    for (int g = 0; g < C::G; ++g) {
      const uint32_t lg = qba_byte_of(g, w0, w1, w2, w3);
#pragma nounroll
      for (int k = g + 1; k < C::G; ++k, ++pi)
        if (lg == qba_byte_of(k, w0, w1, w2, w3)) atomicAdd(&c[pi], 1u);
    }
  }
}

// Samplers of one entry into the byte layout
enum { QBA_S_GENERAL = 0, QBA_S_FAST = 1, QBA_S_CLOSED = 2 };

template <int NP, int SAMP>
__device__ __forceinline__ void qba_entry_d(uint64_t e, uint32_t k0, uint32_t k1,
                                            const QbaProgramSet *__restrict__ ps,
                                            const uint64_t *pat, const uint64_t *apat,
                                            const uint64_t *thr, const uint32_t *pl,
                                            uint32_t (&D)[CF<NP>::ND]) {
  if constexpr (SAMP == QBA_S_CLOSED) {
    qba_closed_entry<NP>(e, k0, k1, pl, D);
  } else if constexpr (SAMP == QBA_S_FAST) {
    qba_out_to_d<NP>(qba_sample_entry_fast<NP>(e, k0, k1, ps->prog[1].perm_t, ps->prog[0].table_len, pat), D);
  } else {
    qba_out_to_d<NP>(qba_sample_entry<NP>(e, k0, k1, ps, pat, apat, thr), D);
  }
}

// Sample one quad (entries [c0, c0+4) of the launch) into the byte layout.
template <int NP, int SAMP, bool TAIL, int PW = QBA_PAIRWISE>
__device__ __forceinline__ void qba_sample_quad(uint32_t c0, int valid, uint64_t first, uint32_t k0,
                                                uint32_t k1, const QbaProgramSet *__restrict__ ps,
                                                const uint64_t *pat, const uint64_t *apat,
                                                const uint64_t *thr, const uint32_t *pl,
                                                uint32_t (&D)[4][CF<NP>::ND]) {
  constexpr int ND = CF<NP>::ND;
  if constexpr (SAMP == QBA_S_CLOSED && !TAIL) {
    // PW: each pair's table reads and finish before the next pair's Philox
    // (fewer live VGPRs: the 8-wave list kernel); else the quad's two Philox
    // blocks interleaved (more ILP: the deferred kernel's low-occupancy step)
    if (PW && !(first & 1)) {
      const uint32_t phi = (uint32_t)(first >> 33);
      const uint32_t plo = (uint32_t)(first >> 1) + (c0 >> 1);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        QbaClosed cl[2];
        const uint64_t p = ((uint64_t)phi << 32) | (uint64_t)(plo + (uint32_t)jp);
        // the 20 round keys loop-invariant in SGPRs (SGPR budget allows them
        // since round 5: 108 instead of 158 SALU per thread-step, cycles -1 %,
        // profiles/r5/keys_sgpr)
        const QbaU4 x = qba_philox_k<false>(plo + (uint32_t)jp, phi, 0u, 0u, k0, k1);
        qba_closed_rank<NP>(x.x, x.y, p, 0u, k0, k1, cl[0]);
        qba_closed_rank<NP>(x.z, x.w, p, 1u, k0, k1, cl[1]);
        uint4 A[2];
        uint2 sB[2];
        uint32_t sC[2];
#pragma unroll
        for (int j = 0; j < 2; ++j) qba_closed_tables<NP>(cl[j].rank, pl, A[j], sB[j], sC[j]);
#pragma unroll
        for (int j = 0; j < 2; ++j) qba_closed_finish<NP>(cl[j], A[j], sB[j], sC[j], D[2 * jp + j]);
      }
      return;
    }
    if (!(first & 1)) {  // wave-uniform: the quad is two whole pairs
      QbaClosed cl[4];
      // A launch never crosses a multiple of 2^33 entries (dispatch splits
      // there), so the pair counter's high word is the launch's and the low
      // word never carries: p_hi stays in an SGPR, Philox's round 1 and half
      // of round 2 are scalar.
      const uint32_t phi = (uint32_t)(first >> 33);
      const uint32_t plo = (uint32_t)(first >> 1) + (c0 >> 1);
#pragma unroll
      for (int jp = 0; jp < 2; ++jp) {
        const uint64_t p = ((uint64_t)phi << 32) | (uint64_t)(plo + (uint32_t)jp);
        const QbaU4 x = qba_philox(plo + (uint32_t)jp, phi, 0u, 0u, k0, k1);
        qba_closed_rank<NP>(x.x, x.y, p, 0u, k0, k1, cl[2 * jp]);
        qba_closed_rank<NP>(x.z, x.w, p, 1u, k0, k1, cl[2 * jp + 1]);
      }
      uint4 A[4];
      uint2 sB[4];
      uint32_t sC[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) qba_closed_tables<NP>(cl[j].rank, pl, A[j], sB[j], sC[j]);
#pragma unroll
      for (int j = 0; j < 4; ++j) qba_closed_finish<NP>(cl[j], A[j], sB[j], sC[j], D[j]);
      return;
    }
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (j < valid) {
      qba_entry_d<NP, SAMP>(first + c0 + j, k0, k1, ps, pat, apat, thr, pl, D[j]);
    } else {
#pragma unroll
      for (int i = 0; i < ND; ++i) D[j][i] = 0;
    }
  }
}

// Every value of a quad of entries < W?  One OR over the quad's transposed
// row words (about 2 VALU per entry) instead of a range test per entry; a
// wave with any out-of-range value takes the per-entry test.
template <int NP>
__device__ __forceinline__ bool qba_rows_in_range(const uint32_t *row) {
  using C = QCfg<NP>;
  uint32_t o = 0;
#pragma unroll
  for (int g = 0; g < C::G; ++g) o |= row[g];
  return !__any((o & (0xffu & ~(uint32_t)(C::W - 1)) * 0x01010101u) != 0u);  // wave-uniform
}

template <int NP>
__device__ __forceinline__ void qba_count_quad(const uint32_t (&D)[4][CF<NP>::ND], int valid,
                                               uint32_t *hist, const uint32_t *row) {
  const uint32_t one = 0x00010001u;
  if (qba_rows_in_range<NP>(row)) {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < valid) qba_count_d<NP>(D[j], one, hist, true);
  } else {
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < valid) qba_count_d<NP>(D[j], one, hist, false);
  }
}

// ---------------------------------------------------------------------------
// Wave-level Q-entry queue: only Q entries are counted, so with
// per-entry counting half the lanes of every count instruction idle.  Each
// wave appends its Q entries (byte-layout words, SoA in LDS) to a ring of
// QBA_QCAP slots and counts them 64 at a time with every lane busy.  All
// queue state is wave-uniform and pushes / drains run with the full wave
// (the callers keep exec full), so no entry is lost or counted twice.
// ---------------------------------------------------------------------------
#define QBA_QCAP 128  // ring slots per wave (two drains' worth)
// L0 != L1 (tfg.py:327) for an active lane: am = 0xff on active lanes, 0 on
// the idle lanes of the last step (one v_bitop3 + compare straight into VCC)
template <int NP>
__device__ __forceinline__ bool qba_isq_d(const uint32_t (&D)[CF<NP>::ND], uint32_t am = 0xffu) {
  return ((D[0] ^ (D[0] >> 8)) & am) != 0u;
}
struct QbaWaveQ {
  uint32_t base;      // LDS byte address of this wave's ring [ND][QBA_QCAP] words (aligned to 4 QBA_QCAP B)
  uint32_t tail, qn;  // wave-uniform: first queued slot (not reduced mod QBA_QCAP), queued entries
  uint32_t hoff;      // LDS byte address of the histogram, kept in a VGPR (see qba_count_d)
};

// LDS byte address of ring slot s (any integer: taken mod QBA_QCAP); the
// ring's alignment makes the slot bits an OR into the base
__device__ __forceinline__ uint32_t qba_q_addr(const QbaWaveQ &q, uint32_t s) {
  return ((s & (QBA_QCAP - 1)) << 2) | q.base;
}
__device__ __forceinline__ qba_lds_u32 *qba_lds(uint32_t addr) {
  return reinterpret_cast<qba_lds_u32 *>(static_cast<uintptr_t>(addr));
}

// The queue area starts after the histogram, aligned to one ring (the host
// sizes the launch's LDS with QBA_QCAP * 4 bytes of slack for it).
template <int NP>
__device__ __forceinline__ uint32_t qba_queue_base(uint32_t *hist) {
  const uint32_t h = (uint32_t)(uintptr_t)(qba_lds_u32 *)hist + ((QCfg<NP>::NBP + 3) & ~3) * 4;
  return (h + QBA_QCAP * 4 - 1) & ~(uint32_t)(QBA_QCAP * 4 - 1);
}

// Count the nv (<= 64) oldest queued entries, one per lane.  TRUSTED: the
// values were produced by this kernel's sampler, masked to nq bits, so
// Cond2's range test cannot fail and is skipped (check-only launches keep it).
template <int NP, bool TRUSTED>
__device__ __forceinline__ void qba_q_drain(QbaWaveQ &q, uint32_t *hist, uint32_t nv) {
  constexpr int ND = CF<NP>::ND;
  const uint32_t lane = __lane_id();
  const uint32_t a = qba_q_addr(q, q.tail + lane);
  uint32_t D[ND];
  // a draining wave issues at raised priority: its queue reads, atomics and
  // address VALU go ahead of the sampling waves', so the LDS queue it feeds
  // drains sooner (745 k -> 727-729 k cycles per launch, window -2.5 %,
  // profiles/r3/r3k/drain_priority_ab.txt)
  __builtin_amdgcn_s_setprio(2);
#pragma unroll
  for (int i = 0; i < ND; ++i) D[i] = *qba_lds(a + i * QBA_QCAP * 4);
  if (nv >= 64 || lane < nv) qba_count_d<NP>(D, 0x00010001u, hist, TRUSTED, true, q.hoff);
  __builtin_amdgcn_s_setprio(0);
  q.tail += nv;
  q.qn -= nv;
}

// Append the lanes' entries with isq set (in lane order) and count a full
// batch of 64 as soon as one is queued.  Slot = tail + qn + the number of
// queued lanes below this one (mbcnt adds the base for free).
template <int NP, bool TRUSTED>
__device__ __forceinline__ void qba_q_push(QbaWaveQ &q, const uint32_t (&D)[CF<NP>::ND], bool isq,
                                           uint32_t *hist) {
  constexpr int ND = CF<NP>::ND;
  const uint64_t m = __ballot(isq);
  // mbcnt from 0 and the wave-uniform base added with the slot-to-byte shift
  // (one v_add_lshl_u32): no v_mov of the base into a VGPR per push
  const uint32_t mb = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (isq) {
    const uint32_t a = (((mb + q.tail + q.qn) << 2) & (uint32_t)(QBA_QCAP * 4 - 1)) | q.base;
#pragma unroll
    for (int i = 0; i < ND; ++i) *qba_lds(a + i * QBA_QCAP * 4) = D[i];
  }
  q.qn += (uint32_t)__popcll(m);
  if (q.qn >= 64) qba_q_drain<NP, TRUSTED>(q, hist, 64u);
}

// ---------------------------------------------------------------------------
// Pair-bin counting (CNT = 1: the fused n = 11 kernel, qba_k_lists MODE 1).
// The classic histogram takes one ds_add_u32 per counted group per Q entry
// (11 at n = 11, ~3.5-way bank conflicts each).  Here one atomic counts TWO
// groups: the bin of a pair (g, h) is (u, L_g, L_h), u = L1, held as an 8-bit
// lane of a dword:
//   array A [x_h][u][x_g] dwords (16 KB): lane 0 = pair (2,3), 1 = (4,5),
//                                         2 = (6,7), 3 = (8,9);
//   array B, same indexing (16 KB):       lane 0 = pair (10,11); lanes 1-3
//     (a 24-bit counter, added as 1 << 8) hold group 0 at x_h = u, and the
//     equal-pair bins C[u][k] at x_g = k & 15, x_h = u ^ (1 + (k >> 4)).
// The byte address of bin (u, x_g, x_h) is 4 x_g + 64 u + 1024 x_h: with
// E = values << 2 (byte g = 4 L_g) a 16-bit half of E IS 4 x_g + 1024 x_h
// for the groups of that half, so each address is ONE v_add_u32 with an SDWA
// word select onto the entry's row base A + 64 u -- as cheap as the classic
// per-group address -- and 6 atomics count the 11 groups.  The queue holds an
// entry as 8 B (c0 = groups 0-3 | groups 4-7 << 4, c1 = groups 8-11): one
// ds_write_b64 per push and one ds_read_b64 per drain instead of 3 + 3.
//
// An 8-bit lane can wrap.  Every Q entry adds exactly one count to every lane
// and to group 0, so per workgroup each lane's total equals group 0's total
// (24 bits, exact: a launch gives a workgroup < 2^24 entries) unless a lane
// wrapped: a wrap loses 256 from its lane and carries at most 1 into the next
// lane up, so some lane's total then differs from group 0's (the lowest
// wrapped lane is short by 255 or 256 net, and a lane can only gain what the
// lane below it lost; B's lane 0 carries into group 0's counter, raising its
// total, never the lane's).  The flush compares the totals and a workgroup
// that finds a mismatch recounts its own entries from the rows it stored,
// with the classic 32-bit bins (qba_lists_body) -- exact in every case.
// The launcher keeps a workgroup at <= QBA_PB_BUDGET entries per launch, so
// for sampled lists a wrap needs a bin ~18 sigma above its mean and never
// happens in practice (tests force it through qba_test_set_knobs' list_grid).
// ---------------------------------------------------------------------------
#define QBA_PB_BUDGET (1u << 18)  // entries per workgroup per launch (wrap-free in practice)
#define QBA_PB_FORCED_LOG2 23     // entries per workgroup (log2) under the tests' list_grid knob
// group 0's total sits in 24-bit lanes: every workgroup must count < 2^24 entries
static_assert(QBA_PB_BUDGET < (1u << 24) && QBA_PB_FORCED_LOG2 < 24, "pair-bin group-0 total is 24 bits");
struct QbaPB {
  static constexpr int WORDS = 8192;       // A [4096] then B [4096]
  static constexpr int BOFF = 4096;        // B, in words
  static constexpr int MISC = 8;           // after B: lane totals [0..4], group 0 total [5]
  static constexpr int AREA = WORDS + MISC;
  static constexpr int QSLOT = 8;          // queue bytes per entry
};
// the kernels that count with pair bins: the fused closed-form n = 11 kernel
// and the n = 11 check of nibble rows (every value < 16 = w, so no range test)
template <int NP, int MODE, int SAMP, int PK>
struct QbaUsePB {
  static constexpr bool value =
      NP == 11 && ((MODE == 1 && SAMP == QBA_S_CLOSED) || (MODE == 2 && PK == 1));
};

// base + 16-bit half h of x in one VALU op (v_add_u32 with an SDWA word select)
__device__ __forceinline__ uint32_t qba_add_word(uint32_t base, uint32_t x, int h) {
  uint32_t r;
  if (h == 0)
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_0" : "=v"(r) : "v"(base), "v"(x));
  else
    asm("v_add_u32_sdwa %0, %1, %2 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "=v"(r) : "v"(base), "v"(x));
  return r;
}

__device__ __forceinline__ void qba_lds_add(uint32_t addr, uint32_t v) {
  atomicAdd((uint32_t *)qba_lds(addr), v);
}

// Count one Q-correlated entry (c0, c1) into the pair bins; hA = LDS byte
// address of array A.  Values are the sampler's (< 16), so no range test.
template <int NP>
__device__ __forceinline__ void qba_count_pb(uint32_t c0, uint32_t c1, uint32_t hA) {
  static_assert(NP == 11, "pair bins are laid out for n = 11");
  constexpr uint32_t B = QbaPB::BOFF * 4;
  const uint32_t E0 = (c0 << 2) & 0x3c3c3c3cu;  // groups 0-3, x4
  const uint32_t t = c0 >> 2;
  const uint32_t E1 = t & 0x3c3c3c3cu;          // groups 4-7, x4
  const uint32_t E2 = c1 << 2;                  // groups 8-11, x4
  // A + 64 u: u = group 1 sits at bits 6-9 of c0 >> 2, and A is 1-KiB
  // aligned (qba_lists_body), so the base is one v_and_or
  const uint32_t hb = (t & 0x3c0u) | hA;
  qba_lds_add(qba_add_word(hb, E0, 0) + B, 0x100u);      // group 0 at (x_0, u, u), B lanes 1-3
  qba_lds_add(qba_add_word(hb, E0, 1), 0x1u);            // (2,3)   A lane 0
  qba_lds_add(qba_add_word(hb, E1, 0), 0x100u);          // (4,5)   A lane 1
  qba_lds_add(qba_add_word(hb, E1, 1), 0x10000u);        // (6,7)   A lane 2
  qba_lds_add(qba_add_word(hb, E2, 0), 0x1000000u);      // (8,9)   A lane 3
  qba_lds_add(qba_add_word(hb, E2, 1) + B, 0x1u);        // (10,11) B lane 0
  // Cond3 (tfg.py:96-98) on every counted entry: its 12 values are pairwise
  // distinct iff the union of their 16-bit one-hots has 12 bits.  Each
  // v_pk_lshlrev_b16 makes two one-hots from the low nibbles of the two
  // halves of its amount: c0 -> groups 0, 2; c0 >> 4 -> 4, 6; c0 >> 8 -> 1,
  // 3; c0 >> 12 -> 5, 7; c1 -> 8, 10; c1 >> 8 -> 9, 11.
  const uint32_t one = 0x00010001u;
  const uint32_t s4 = c0 >> 4;
  // the union as two all-VGPR v_bitop3_b32 (a | b | c) and one v_or_b32, the
  // forms gfx950 issues at the full rate, instead of v_or + two v_or3_b32
  // (tools/exp/valu_mix2.hip; the same cycles per launch, the driver's window
  // -3 % in the 300-launch traces of profiles/r6/ab_cond3_bitop3)
  uint32_t U = __builtin_amdgcn_bitop3_b32(qba_pk_onehot(c0, one), qba_pk_onehot(s4, one),
                                           qba_pk_onehot(c0 >> 8, one), 0xFE);
  U = __builtin_amdgcn_bitop3_b32(U, qba_pk_onehot(s4 >> 8, one), qba_pk_onehot(c1, one), 0xFE);
  U |= qba_pk_onehot(c1 >> 8, one);
  if (__popc(qba_fold16(U)) != QCfg<NP>::G) {  // some pair collides: exact slow path
    // C[u][k] for every equal pair k = pidx(g, h): B lanes 1-3 of the word
    // (x_g = k & 15, u, x_h = u ^ (1 + k / 16)), a word no Q entry's group 0
    // uses (x_h != u; qba_pb_flush reads them back)
    const uint32_t w0 = c0 & 0x0f0f0f0fu, w1 = s4 & 0x0f0f0f0fu, w2 = c1;
    const uint32_t u = __builtin_amdgcn_ubfe(c0, 8, 4);
    int k = 0;
#pragma nounroll
    for (int g = 0; g < QCfg<NP>::G; ++g) {
      const uint32_t lg = qba_byte_of(g, w0, w1, w2, 0u);
#pragma nounroll
      for (int h = g + 1; h < QCfg<NP>::G; ++h, ++k)
        if (lg == qba_byte_of(h, w0, w1, w2, 0u))
          qba_lds_add(hA + B + 4 * (uint32_t)((k & 15) + 16 * u + 256 * (u ^ (1 + (k >> 4)))), 0x100u);
    }
  }
}

// the queue's 8-B form of an entry in the byte layout (values < 16)
template <int NP>
__device__ __forceinline__ uint2 qba_pb_pack(const uint32_t (&D)[CF<NP>::ND]) {
  return make_uint2(D[0] | (D[1] << 4), D[2]);
}

// The pair-bin queue is LINEAR: slots [0, qn) of the wave's 128-slot area
// hold the queued entries.  A push writes slot qn + (queued lanes below this
// one): ONE v_add_lshl_u32 (the wave's base / 8 rides in the SGPR sum); a
// drain counts slots [0, nv), one per lane at a loop-invariant address, then
// moves the leftover (< 64 entries) down to slot 0 with one read (offset
// 512) and one write per leftover lane.
template <int NP>
__device__ __forceinline__ void qba_q_drain_pb(QbaWaveQ &q, uint32_t nv) {
  const uint32_t lane = __lane_id();
  typedef uint32_t v2u __attribute__((ext_vector_type(2)));
  typedef __attribute__((address_space(3))) v2u lds_v2u;
  uint32_t a;  // base + 8 lane in one op
  asm("v_lshl_add_u32 %0, %1, 3, %2" : "=v"(a) : "v"(lane), "s"(q.base));
  const v2u c = *reinterpret_cast<lds_v2u *>(static_cast<uintptr_t>(a));
  __builtin_amdgcn_s_setprio(2);  // as qba_q_drain
  if (nv >= 64 || lane < nv) qba_count_pb<NP>(c.x, c.y, q.hoff);
  __builtin_amdgcn_s_setprio(0);
  q.qn -= nv;
  if (q.qn) {  // wave-uniform: the leftover of a full drain (nv = 64)
    if (lane < q.qn) {
      const v2u m = *reinterpret_cast<lds_v2u *>(static_cast<uintptr_t>(a + 512u));
      *reinterpret_cast<lds_v2u *>(static_cast<uintptr_t>(a)) = m;
    }
  }
}

// The lanes whose entry is Q-correlated (L0 != L1, tfg.py:327: byte 0 vs byte
// 1 of word 0 of the byte layout) among the active lanes `act`: one SDWA
// v_cmp, then an s_and -- the last writer of the mask is the scalar unit.
__device__ __forceinline__ uint64_t qba_isq_mask(uint32_t w0, uint64_t act) {
  uint64_t m;
  asm("v_cmp_ne_u32_sdwa %0, %1, %1 src0_sel:BYTE_0 src1_sel:BYTE_1\n\ts_and_b64 %0, %0, %2"
      : "=&s"(m) : "v"(w0), "s"(act));
  return m;
}

// Push the entries of the lanes in m (a lane mask, qba_isq_mask)
template <int NP>
__device__ __forceinline__ void qba_q_push_pb_m(QbaWaveQ &q, const uint32_t (&D)[CF<NP>::ND], uint64_t m) {
  const uint32_t mb = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (__builtin_amdgcn_inverse_ballot_w64(m)) {
    uint32_t a;  // (mb + qn + base / 8) * 8 in one op
    asm("v_add_lshl_u32 %0, %1, %2, 3" : "=v"(a) : "v"(mb), "s"(q.qn + (q.base >> 3)));
    const uint2 c = qba_pb_pack<NP>(D);
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    v2u cv;
    cv.x = c.x;
    cv.y = c.y;
    *reinterpret_cast<__attribute__((address_space(3))) v2u *>(static_cast<uintptr_t>(a)) = cv;
  }
  q.qn += (uint32_t)__popcll(m);
  if (q.qn >= 64) qba_q_drain_pb<NP>(q, 64u);
}

template <int NP>
__device__ __forceinline__ void qba_q_push_pb(QbaWaveQ &q, const uint32_t (&D)[CF<NP>::ND], bool isq) {
  const uint64_t m = __ballot(isq);
  const uint32_t mb = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
  if (isq) {
    uint32_t a;  // (mb + qn + base / 8) * 8 in one op (the compiler splits it into three)
    asm("v_add_lshl_u32 %0, %1, %2, 3" : "=v"(a) : "v"(mb), "s"(q.qn + (q.base >> 3)));
    const uint2 c = qba_pb_pack<NP>(D);
    typedef uint32_t v2u __attribute__((ext_vector_type(2)));
    v2u cv;
    cv.x = c.x;
    cv.y = c.y;
    *reinterpret_cast<__attribute__((address_space(3))) v2u *>(static_cast<uintptr_t>(a)) = cv;
  }
  q.qn += (uint32_t)__popcll(m);
  if (q.qn >= 64) qba_q_drain_pb<NP>(q, 64u);
}

// Push (the wave queue) / count one entry directly (tails) with the counting
// scheme CNT (0: classic 32-bit bins in `hist`, 1: pair bins, hist = array A).
template <int NP, bool TRUSTED, int CNT>
__device__ __forceinline__ void qba_push(QbaWaveQ &q, const uint32_t (&D)[CF<NP>::ND], bool isq, uint32_t *hist) {
  if constexpr (CNT == 1)
    qba_q_push_pb<NP>(q, D, isq);
  else
    qba_q_push<NP, TRUSTED>(q, D, isq, hist);
}
template <int NP, int CNT>
__device__ __forceinline__ void qba_count_one(const uint32_t (&D)[CF<NP>::ND], uint32_t *hist) {
  if constexpr (CNT == 1) {
    if ((D[0] & 0xffu) == ((D[0] >> 8) & 0xffu)) return;  // not Q-correlated (tfg.py:327)
    const uint2 c = qba_pb_pack<NP>(D);
    qba_count_pb<NP>(c.x, c.y, (uint32_t)(uintptr_t)(qba_lds_u32 *)hist);
  } else {
    qba_count_d<NP>(D, 0x00010001u, hist, true);
  }
}

// One thread-step over QPT consecutive quads: entries [c0, c0 + 4 QPT) of the
// launch (columns of `lists`).  Each list row is stored / loaded as one
// 4*QPT-byte vector per thread (16 B at QPT = 4: a wave moves 1 KiB per row).
// MODE 0: sample -> lists;  MODE 1: sample -> lists + counts;  MODE 2: lists -> counts
// TAIL (QPT = 1 only): the last, partial quad, byte by byte.
template <int NP, int MODE, int SAMP, int QPT, bool TAIL, bool WQ = false, int CNT = 0, int PW = QBA_PAIRWISE>
__device__ __forceinline__ void qba_step(uint32_t c0, uint32_t count, uint64_t first, uint32_t k0,
                                         uint32_t k1, const QbaProgramSet *__restrict__ ps,
                                         const uint64_t *pat, const uint64_t *apat,
                                         const uint64_t *thr, const uint32_t *pl,
                                         uint8_t *__restrict__ lists, uint64_t ld, uint32_t *hist,
                                         QbaWaveQ *wq = nullptr, bool act = true) {
  using C = QCfg<NP>;
  constexpr int ND = CF<NP>::ND;
  static_assert(QPT == 1 || QPT == 2 || QPT == 4, "QPT");
  static_assert(!TAIL || QPT == 1, "tail quads are single");
  static_assert(CNT == 0 || MODE == 1, "pair bins count the fused kernel's own lists only");
  typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));
  typedef uint32_t u32x2 __attribute__((ext_vector_type(2)));
  using V = typename std::conditional<QPT == 4, u32x4, typename std::conditional<QPT == 2, u32x2, uint32_t>::type>::type;
  const int valid = !TAIL ? 4 : ((count - c0) >= 4 ? 4 : (int)(count - c0));
  uint32_t row[QPT][4 * ND];
  uint32_t D[4][ND];
  const uint32_t am = act ? 0xffu : 0u;
  if constexpr (MODE == 2) {
#pragma unroll
    for (int k = 0; k < QPT; ++k)
#pragma unroll
      for (int g = 0; g < 4 * ND; ++g) row[k][g] = 0;
    if (!TAIL && act) {
#pragma unroll
      for (int g = 0; g < C::G; ++g) {
        const V v = __builtin_nontemporal_load(reinterpret_cast<const V *>(lists + (uint64_t)g * ld + c0));
        const uint32_t *pv = reinterpret_cast<const uint32_t *>(&v);
#pragma unroll
        for (int k = 0; k < QPT; ++k) row[k][g] = pv[k];
      }
    } else if (TAIL) {
      for (int g = 0; g < C::G; ++g)
        for (int j = 0; j < valid; ++j) row[0][g] |= (uint32_t)lists[(uint64_t)g * ld + c0 + j] << (8 * j);
    }
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
#pragma unroll
      for (int i = 0; i < ND; ++i)
        qba_t4(row[k][4 * i], row[k][4 * i + 1], row[k][4 * i + 2], row[k][4 * i + 3], D[0][i],
               D[1][i], D[2][i], D[3][i]);
      if constexpr (WQ) {  // the caller's queue (never null)
#pragma unroll
        for (int j = 0; j < 4; ++j) qba_q_push<NP, MODE == 1>(*wq, D[j], qba_isq_d<NP>(D[j], am), hist);
      } else {
        qba_count_quad<NP>(D, valid, hist, row[k]);
      }
    }
  } else {
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
      qba_sample_quad<NP, SAMP, TAIL, PW>(c0 + 4 * k, valid, first, k0, k1, ps, pat, apat, thr, pl, D);
#pragma unroll
      for (int i = 0; i < ND; ++i)
        qba_t4(D[0][i], D[1][i], D[2][i], D[3][i], row[k][4 * i], row[k][4 * i + 1],
               row[k][4 * i + 2], row[k][4 * i + 3]);
      if constexpr (MODE == 1) {
        if constexpr (WQ) {  // the caller's queue (never null)
          // L0 != L1 (tfg.py:327) of the quad's 4 entries at once: byte j of
          // row 0 XOR row 1 is nonzero iff entry j is Q-correlated
          const uint32_t xq = (row[k][0] ^ row[k][1]) & (act ? 0xffffffffu : 0u);
#pragma unroll
          for (int j = 0; j < 4; ++j)
            qba_push<NP, MODE == 1, CNT>(*wq, D[j], (xq & (0xffu << (8 * j))) != 0u, hist);
        } else if constexpr (CNT == 1) {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < valid) qba_count_one<NP, 1>(D[j], hist);
        } else {
          qba_count_quad<NP>(D, valid, hist, row[k]);
        }
      }
    }
    if (!TAIL && act)
    {
#pragma unroll
      for (int g = 0; g < C::G; ++g) {
        V v;
        uint32_t *pv = reinterpret_cast<uint32_t *>(&v);
#pragma unroll
        for (int k = 0; k < QPT; ++k) pv[k] = row[k][g];
        // row base opaque in SGPRs (an empty asm: no instruction is emitted),
        // so the store is `global_store v_c0, v_data, s[row]` with a 32-bit
        // lane offset -- otherwise the compiler shares lists + c0 as a 64-bit
        // VGPR and pays a 64-bit VALU add per row
        uint64_t rb = reinterpret_cast<uint64_t>(lists) + (uint64_t)g * ld;
        asm("" : "+s"(rb));
        typedef __attribute__((address_space(1))) V GV;  // global, not flat
        GV *dst = reinterpret_cast<GV *>(rb + c0);
        // the rows are streamed out once: nontemporal stores move the 12 rows of
        // 1.25e8 entries in 0.313 ms instead of 0.356 (tools/ubench/stores2)
        __builtin_nontemporal_store(v, dst);
      }
    } else if (TAIL) {
      for (int g = 0; g < C::G; ++g)
        for (int j = 0; j < valid; ++j) lists[(uint64_t)g * ld + c0 + j] = (uint8_t)(row[0][g] >> (8 * j));
    }
  }
}

// The same thread-step over NIBBLE rows (qba.h, "packed lists"): byte b of
// row g holds columns 2b (low nibble) and 2b+1 (high nibble), half the bytes
// of the byte layout.  Every value is < w <= 16, so two entries' byte-layout
// words fold into one word -- D[2p] | D[2p+1] << 4, byte g' = the packed pair
// of group 4i+g' -- BEFORE the transpose: one 4x4 transpose per 8 entries
// (QPT = 2, one 4-B store per row) instead of two, and half the HBM writes,
// which keeps the chip's clock up in the driver's cold window
// (profiles/r3/ab32_microopts_and_stores.txt: 12-row packed stores 375-381 us vs 421-424 us).
// QPT = 1 (unaligned starts, the tail quads): 2 bytes per row, stored as bytes
// (a chunk may start at an odd byte).  MODE 2 reads the same layout; an
// unpacked quad's entries come out permuted (counting is order-free).
template <int NP, int MODE, int SAMP, int QPT, bool TAIL, bool WQ = false, int CNT = 0, int PW = QBA_PAIRWISE>
__device__ __forceinline__ void qba_step_pk(uint32_t c0, uint32_t count, uint64_t first, uint32_t k0,
                                            uint32_t k1, const QbaProgramSet *__restrict__ ps,
                                            const uint64_t *pat, const uint64_t *apat,
                                            const uint64_t *thr, const uint32_t *pl,
                                            uint8_t *__restrict__ lists, uint64_t ld, uint32_t *hist,
                                            QbaWaveQ *wq, bool act) {
  using C = QCfg<NP>;
  constexpr int ND = CF<NP>::ND;
  static_assert(QPT == 1 || QPT == 2, "packed rows: QPT 1 or 2");
  static_assert(!TAIL || QPT == 1, "tail quads are single");
  static_assert(CNT == 0 || MODE != 0, "pair bins count");
  static_assert(C::W <= 16, "a value must fit a nibble");
  typedef __attribute__((address_space(1))) uint32_t GU;
  const int valid = !TAIL ? 4 : ((count - c0) >= 4 ? 4 : (int)(count - c0));
  const uint64_t cb = c0 >> 1;  // byte column of the step's first entry
  uint32_t D[4][ND];
  if constexpr (MODE == 2) {
    uint32_t row[QPT][4 * ND];
#pragma unroll
    for (int k = 0; k < QPT; ++k)
#pragma unroll
      for (int g = 0; g < 4 * ND; ++g) row[k][g] = 0;
    if (!TAIL && act) {
#pragma unroll
      for (int g = 0; g < C::G; ++g) {
        if constexpr (QPT == 2) {
          uint64_t rb = reinterpret_cast<uint64_t>(lists) + (uint64_t)g * ld;
          asm("" : "+s"(rb));
          const uint32_t v = __builtin_nontemporal_load(reinterpret_cast<const GU *>(rb + cb));
          row[0][g] = v & 0x0f0f0f0fu;         // columns 0, 2, 4, 6
          row[1][g] = (v >> 4) & 0x0f0f0f0fu;  // columns 1, 3, 5, 7
        } else {
          const uint8_t *r = lists + (uint64_t)g * ld + cb;
          const uint32_t h = (uint32_t)r[0] | ((uint32_t)r[1] << 8);
          row[0][g] = (h & 0x0f0fu) | ((h & 0xf0f0u) << 12);  // columns 0, 2, 1, 3
        }
      }
    } else if (TAIL) {
      for (int g = 0; g < C::G; ++g)
        for (int j = 0; j < valid; ++j)
          row[0][g] |= (uint32_t)((lists[(uint64_t)g * ld + cb + (j >> 1)] >> (4 * (j & 1))) & 15) << (8 * j);
    }
    const uint32_t am = act ? 0xffu : 0u;
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
#pragma unroll
      for (int i = 0; i < ND; ++i)
        qba_t4(row[k][4 * i], row[k][4 * i + 1], row[k][4 * i + 2], row[k][4 * i + 3], D[0][i],
               D[1][i], D[2][i], D[3][i]);
      if constexpr (WQ) {  // the caller's queue (never null)
#pragma unroll
        for (int j = 0; j < 4; ++j) qba_push<NP, false, CNT>(*wq, D[j], qba_isq_d<NP>(D[j], am), hist);
      } else if constexpr (CNT == 1) {
#pragma unroll
        for (int j = 0; j < 4; ++j)
          if (j < (TAIL ? valid : 4)) qba_count_one<NP, 1>(D[j], hist);
      } else {
        qba_count_quad<NP>(D, TAIL ? valid : 4, hist, row[k]);
      }
    }
  } else {
    uint32_t Dp[2 * QPT][ND];  // pair p: entries 2p, 2p+1 of the step
    const uint32_t am = act ? 0xffu : 0u;
    const uint64_t actm = __ballot(act);  // the step's active lanes
#pragma unroll
    for (int k = 0; k < QPT; ++k) {
      qba_sample_quad<NP, SAMP, TAIL, PW>(c0 + 4 * k, valid, first, k0, k1, ps, pat, apat, thr, pl, D);
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        Dp[2 * k][i] = D[0][i] | (D[1][i] << 4);
        Dp[2 * k + 1][i] = D[2][i] | (D[3][i] << 4);
      }
      if constexpr (MODE == 1) {
        if constexpr (WQ) {  // the caller's queue (never null)
          if constexpr (CNT == 1) {
            // L0 != L1 (tfg.py:327) of each entry: one SDWA compare of byte 0
            // with byte 1 of its word 0, the step's active lanes ANDed in on
            // the scalar unit
#pragma unroll
            for (int j = 0; j < 4; ++j) qba_q_push_pb_m<NP>(*wq, D[j], qba_isq_mask(D[j][0], actm));
          } else {
            // ... of a pair at once: nibble 0 / 1 of (byte 0 ^ byte 1) of its
            // packed word 0 is entry 2p / 2p+1's test
#pragma unroll
            for (int p = 0; p < 2; ++p) {
              const uint32_t w0 = Dp[2 * k + p][0];
              const uint32_t x = (w0 ^ (w0 >> 8)) & am;
              qba_push<NP, true, CNT>(*wq, D[2 * p], (x & 0x0fu) != 0u, hist);
              qba_push<NP, true, CNT>(*wq, D[2 * p + 1], x > 0x0fu, hist);
            }
          }
        } else {
#pragma unroll
          for (int j = 0; j < 4; ++j)
            if (j < valid) qba_count_one<NP, CNT>(D[j], hist);
        }
      }
    }
    if (!TAIL && act) {
      uint64_t rbl = 0;  // the running row base
      (void)rbl;
#pragma unroll
      for (int i = 0; i < ND; ++i) {
        uint32_t r[4];
        if constexpr (QPT == 2)
          qba_t4(Dp[0][i], Dp[1][i], Dp[2][i], Dp[3][i], r[0], r[1], r[2], r[3]);
        else
          qba_t4(Dp[0][i], Dp[1][i], 0u, 0u, r[0], r[1], r[2], r[3]);
#pragma unroll
        for (int gg = 0; gg < 4; ++gg) {
          const int g = 4 * i + gg;
          if (g >= C::G) continue;
          // row base opaque in SGPRs, 32-bit lane offset (as qba_step)
          // one running row pointer (s_add_u32 / s_addc_u32 per row) instead
          // of n+1 loop-invariant 64-bit bases
          if (g == 0) {
            rbl = reinterpret_cast<uint64_t>(lists);
            asm volatile("" : "+s"(rbl));
          } else {
            rbl += ld;
            asm volatile("" : "+s"(rbl));
          }
          const uint64_t rb = rbl;
          if constexpr (QPT == 2) {
            __builtin_nontemporal_store(r[gg], reinterpret_cast<GU *>(rb + cb));
          } else if (!((reinterpret_cast<uintptr_t>(lists) | ld) & 1)) {  // uniform: rows 2-byte aligned (cb is even)
            typedef __attribute__((address_space(1))) uint16_t GH;
            *reinterpret_cast<GH *>(rb + cb) = (uint16_t)r[gg];
          } else {
            uint8_t *d = reinterpret_cast<uint8_t *>(rb + cb);
            d[0] = (uint8_t)r[gg];
            d[1] = (uint8_t)(r[gg] >> 8);
          }
        }
      }
    } else if (TAIL) {
      // the call's last, partial quad: its bytes (a missing entry's nibble is 0)
      for (int i = 0; i < ND; ++i)
        for (int gg = 0; gg < 4; ++gg) {
          const int g = 4 * i + gg;
          if (g >= C::G) continue;
          for (int b = 0; 2 * b < valid; ++b)
            lists[(uint64_t)g * ld + cb + b] = (uint8_t)(Dp[b][i] >> (8 * gg));
        }
    }
  }
}

template <int NP, int MODE, int SAMP, int QPT, bool TAIL, int PK, bool WQ = false, int CNT = 0, int PW = QBA_PAIRWISE>
__device__ __forceinline__ void qba_step_l(uint32_t c0, uint32_t count, uint64_t first, uint32_t k0,
                                           uint32_t k1, const QbaProgramSet *__restrict__ ps,
                                           const uint64_t *pat, const uint64_t *apat,
                                           const uint64_t *thr, const uint32_t *pl,
                                           uint8_t *__restrict__ lists, uint64_t ld, uint32_t *hist,
                                           QbaWaveQ *wq = nullptr, bool act = true) {
  if constexpr (PK)
    qba_step_pk<NP, MODE, SAMP, QPT, TAIL, WQ, CNT, PW>(c0, count, first, k0, k1, ps, pat, apat, thr, pl, lists, ld, hist, wq, act);
  else
    qba_step<NP, MODE, SAMP, QPT, TAIL, WQ, CNT, PW>(c0, count, first, k0, k1, ps, pat, apat, thr, pl, lists, ld, hist, wq, act);
}

// Stage the program's tables in LDS; returns the histogram base after them.
template <int NP, int MODE, int SAMP, int BS>
__device__ __forceinline__ uint32_t *qba_stage(const QbaProgramSet *__restrict__ ps, uint64_t *lds,
                                               const uint64_t *&pat, const uint64_t *&apat,
                                               const uint64_t *&thr, const uint32_t *&pl) {
  pat = apat = thr = lds;
  pl = reinterpret_cast<const uint32_t *>(lds);
  uint32_t *hist = reinterpret_cast<uint32_t *>(lds);
  if constexpr (MODE != 2 && SAMP == QBA_S_CLOSED) {
    // at a compile-time offset: the loads issue without reading the header
    const uint32_t *src = reinterpret_cast<const uint32_t *>(reinterpret_cast<const char *>(ps) + QBA_PERM_OFF);
    uint32_t *dst = reinterpret_cast<uint32_t *>(lds);
    // 16-B buffer loads, all issued before the first LDS write: one memory
    // round trip per workgroup (the image pads the tables to whole 16-B
    // words, qba_plan_image).  A buffer load past the tables' W4 words returns
    // zero, so every lane loads unconditionally at a 32-bit offset; only the
    // LDS writes are guarded.  (Plain loads with a guard were serialised by
    // the compiler -- load, wait, write, per word -- or went to scratch.)
    constexpr int W4 = (CF<NP>::WORDS + 3) / 4, PER = (W4 + BS - 1) / BS;
    typedef uint32_t v4u __attribute__((ext_vector_type(4)));
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<uint32_t *>(src), (short)0, W4 * 16, 0x00020000);
    v4u v[PER];
#pragma unroll
    for (int k = 0; k < PER; ++k) v[k] = __builtin_amdgcn_raw_buffer_load_b128(rs, (threadIdx.x + k * BS) * 16u, 0, 0);
    // the guarded writes' loads are not sunk into their branches
#pragma unroll
    for (int k = 0; k < PER; ++k) asm volatile("" ::"v"(v[k]));
    uint4 *d4 = reinterpret_cast<uint4 *>(dst);
#pragma unroll
    for (int k = 0; k < PER; ++k)
      if (threadIdx.x + k * BS < W4) d4[threadIdx.x + k * BS] = make_uint4(v[k].x, v[k].y, v[k].z, v[k].w);
    hist = dst + ((CF<NP>::WORDS + 3) & ~3);
  } else if constexpr (MODE != 2) {
    const int T = ps->table_total;
    const uint64_t *tab = reinterpret_cast<const uint64_t *>(reinterpret_cast<const char *>(ps) + ps->tab_off);
    const int ntab = ps->any_nonuniform ? 3 * T : T;
    for (int i = threadIdx.x; i < ntab; i += BS) lds[i] = tab[i];
    apat = lds + T;
    thr = lds + 2 * T;
    hist = reinterpret_cast<uint32_t *>(lds + ((ntab + 1) & ~1));  // 16-B aligned
  }
  return hist;
}

// The outputs of a counting launch start at zero unless the call accumulates:
// the list kernel's workgroup 0 clears them before the reduction adds in.
struct QbaZero {
  int64_t *H, *C, *P, *stats;
  uint32_t flags;  // bit 0: clear H, C, P; bit 1: clear the stats
};
template <int NP>
__device__ __forceinline__ void qba_zero_outputs(const QbaZero &z, int tid, int bs) {
  using C = QCfg<NP>;
  if (z.flags & 1) {
    for (int i = tid; i < C::HB; i += bs) z.H[i] = 0;
    for (int i = tid; i < C::CB; i += bs) z.C[i] = 0;
    for (int i = tid; i < C::W; i += bs) z.P[i] = 0;
  }
  if ((z.flags & 2) && z.stats && tid < C::STATS) z.stats[tid] = 0;
}

// The pair bins' flush: the classic slab row (H [u][g][x] as counted, the
// pair bins C[u][k], the stats) from the marginals of arrays A / B, after the
// wrap test (see QbaPB).  Returns true -- for every thread -- when a lane
// wrapped; the slab row is then left to the caller's recount.  Slab words of
// group 1 and the row padding are not written (the reductions skip them).
template <int NP, int BS>
__device__ __forceinline__ bool qba_pb_flush(uint32_t *hist, uint32_t *row, int t) {
  using C = QCfg<NP>;
  static_assert(BS >= 512, "four roles of 256 threads");
  const uint32_t *A = hist, *Bw = hist + QbaPB::BOFF;
  uint32_t *misc = hist + QbaPB::WORDS;
  uint32_t v[5] = {0u, 0u, 0u, 0u, 0u}, g0 = 0u;
  const int ug = (t & 255) >> 4, xg = t & 15;    // column-sum threads: (u, x)
  const int ur = t & 15, yr = (t & 255) >> 4;    // row-sum threads: (u, y), u fastest
  if (t < 256) {  // groups 2, 4, 6, 8, 10 (x_g of each pair): sums over x_h
    uint32_t s02 = 0u, s13 = 0u, sb = 0u;
    const uint32_t *a = A + xg + 16 * ug, *b = Bw + xg + 16 * ug;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      const uint32_t d = a[256 * k];
      s02 += d & 0x00ff00ffu;
      s13 += (d >> 8) & 0x00ff00ffu;
      sb += b[256 * k] & 0xffu;
    }
    v[0] = s02 & 0xffffu;  // (2,3)
    v[1] = s13 & 0xffffu;  // (4,5)
    v[2] = s02 >> 16;      // (6,7)
    v[3] = s13 >> 16;      // (8,9)
    v[4] = sb;             // (10,11)
    g0 = Bw[xg + 16 * ug + 256 * ug] >> 8;
    // lane totals: summed across the wave first (64 same-address LDS atomics
    // per instruction serialise: +12 us per launch), then one atomic per wave
    uint32_t s6[6] = {v[0], v[1], v[2], v[3], v[4], g0};
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1)
#pragma unroll
      for (int p = 0; p < 6; ++p) s6[p] += __shfl_xor(s6[p], m, 64);
    if ((t & 63) == 0)
#pragma unroll
      for (int p = 0; p < 6; ++p) atomicAdd(&misc[p], s6[p]);
  } else if (t < 512) {  // groups 3, 5, 7, 9, 11 (x_h of each pair): sums over x_g
    uint32_t s02 = 0u, s13 = 0u, sb = 0u;
    const uint4 *a = reinterpret_cast<const uint4 *>(A + 16 * ur + 256 * yr);
    const uint4 *b = reinterpret_cast<const uint4 *>(Bw + 16 * ur + 256 * yr);
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      const uint4 d = a[(k + ur) & 3], e = b[(k + ur) & 3];  // rotated: fewer bank conflicts
      s02 += (d.x & 0x00ff00ffu) + (d.y & 0x00ff00ffu) + (d.z & 0x00ff00ffu) + (d.w & 0x00ff00ffu);
      s13 += ((d.x >> 8) & 0x00ff00ffu) + ((d.y >> 8) & 0x00ff00ffu) + ((d.z >> 8) & 0x00ff00ffu) +
             ((d.w >> 8) & 0x00ff00ffu);
      sb += (e.x & 0xffu) + (e.y & 0xffu) + (e.z & 0xffu) + (e.w & 0xffu);
    }
    v[0] = s02 & 0xffffu;
    v[1] = s13 & 0xffffu;
    v[2] = s02 >> 16;
    v[3] = s13 >> 16;
    v[4] = sb;
  }
  __syncthreads();
  const bool wrap = misc[0] != misc[5] || misc[1] != misc[5] || misc[2] != misc[5] || misc[3] != misc[5] ||
                    misc[4] != misc[5];
  if (wrap) return true;  // workgroup-uniform
  if (t < 256) {
    row[(ug * C::G + 0) * C::WP + xg] = g0;
#pragma unroll
    for (int p = 0; p < 5; ++p) row[(ug * C::G + 2 + 2 * p) * C::WP + xg] = v[p];
  } else if (t < 512) {
#pragma unroll
    for (int p = 0; p < 5; ++p) row[(ur * C::G + 3 + 2 * p) * C::WP + yr] = v[p];
  }
  for (int i = t; i < C::CBL; i += BS) {  // C[u][k]: B lanes 1-3 at (k & 15, u, u ^ (1 + k / 16))
    const int u = i / C::CP, k = i - u * C::CP;
    row[C::HBL + i] = Bw[(k & 15) + 16 * u + 256 * (u ^ (1 + (k >> 4)))] >> 8;
  }
  if (t < C::STATS) row[C::HBL + C::CBL + t] = 0u;  // sampled values are < w
  return false;
}

// Waves per SIMD the list kernels are compiled for.  The closed-form sampler
// runs 2 workgroups of 1024 threads per CU = 8 waves per SIMD (the CDNA4
// maximum): with its quads sampled pair by pair (QBA_PAIRWISE) and the round
// keys / row bases re-derived on the scalar unit (QBA_SGPR_LEAN) it fits the
// 64 VGPRs and the SGPR budget that needs, and the extra waves hide the LDS
// latency of the histogram atomics: -3 % cycles per launch against 6 waves
// of 768 threads (profiles/r3/r3k).  The table samplers (n > 11) need more
// registers and keep the compiler's choice.
#define QBA_LISTS_BOUNDS \
  __attribute__((amdgpu_flat_work_group_size(1, QBA_LBLOCK), amdgpu_waves_per_eu(SAMP == QBA_S_CLOSED ? 8 : 1)))
#define QBA_LISTS_BOUNDS_PB \
  __attribute__((amdgpu_flat_work_group_size(1, QBA_LBLOCK), amdgpu_waves_per_eu(8)))
// PK = 1: nibble rows (qba_step_pk), ld in bytes of packed row.
// The body of the list kernel; its workgroups are those after the first
// `red` (qba_k_lists: 0; qba_k_lists_def: its reduce workgroups).
template <int NP, int MODE, int SAMP, int QPT, int PK, int BS = QBA_LBLOCK, int CNT = 0, int PW = QBA_PAIRWISE>
__device__ __forceinline__ void qba_lists_body(const QbaProgramSet *__restrict__ ps, uint32_t k0, uint32_t k1,
                                               uint64_t first, uint32_t count, uint8_t *__restrict__ lists,
                                               uint64_t ld, uint32_t *__restrict__ slab, QbaZero zero,
                                               uint32_t red, uint32_t tail = 0) {
  using C = QCfg<NP>;
  extern __shared__ __align__(16) uint64_t lds[];
  // list workgroups: [red, gridDim.x - tail) (reduce workgroups of a
  // deferred reduction after them, qba_k_lists_def and
  // qba_k_lists_pbdef)
  const uint32_t bid = blockIdx.x - red, nblk = gridDim.x - red - tail;
  const uint64_t *pat, *apat, *thr;
  const uint32_t *pl;
  uint32_t *hist = qba_stage<NP, MODE, SAMP, BS>(ps, lds, pat, apat, thr, pl);
  if constexpr (CNT) {  // pair bins: array A 1-KiB aligned (qba_count_pb ORs 64 u into its address)
    const uint32_t h = (uint32_t)(uintptr_t)(qba_lds_u32 *)hist;
    hist += (((h + 1023u) & ~1023u) - h) / 4;
  }
  if (MODE != 0) {
    constexpr int NZ = CNT ? QbaPB::AREA : C::NBP;
    for (int i = threadIdx.x; i < NZ; i += BS) hist[i] = 0u;
  }
  __syncthreads();
  const uint32_t nunits = count / (4 * QPT);
  // the grid stride in an SGPR, read once: reloading gridDim in the loop is a
  // scalar load whose s_waitcnt lgkmcnt(0) also drains every LDS atomic the
  // wave has in flight (-2% step time)
  const uint32_t ustride = __builtin_amdgcn_readfirstlane(nblk * BS);
  // unit u of a step: wave-major over the grid (wave w of workgroup b takes
  // units [(w nblk + b) 64, +64)), so a launch with fewer units than threads
  // spreads them over every workgroup instead of filling the first ones;
  // a wave's 64 units stay consecutive (one 256-B / 512-B store per row)
  const uint32_t u0 = ((threadIdx.x >> 6) * nblk + bid) * 64u + (threadIdx.x & 63u);
  // the wave's index in an SGPR: the code after the main loop rebuilds the
  // thread index from it and the lane id instead of keeping threadIdx.x (and
  // what derives from it) live across the loop -- at 64 VGPRs those values
  // were spilled to scratch, and a kernel with scratch waits ~6 us longer for
  // its dispatch after the previous kernel (profiles/r5/slab_event)
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  if constexpr (MODE != 0) {
    QbaWaveQ wq;
    if constexpr (CNT) {  // 8-B slots after the pair bins, each ring aligned to its size
      const uint32_t h = (uint32_t)(uintptr_t)(qba_lds_u32 *)hist + QbaPB::AREA * 4;
      wq.base = __builtin_amdgcn_readfirstlane(((h + QBA_QCAP * 8 - 1) & ~(uint32_t)(QBA_QCAP * 8 - 1)) +
                                               (threadIdx.x >> 6) * (QBA_QCAP * 8));
    } else {
      wq.base = qba_queue_base<NP>(hist) + (threadIdx.x >> 6) * (CF<NP>::ND * QBA_QCAP * 4);
    }
    wq.tail = 0;
    wq.qn = 0;
    wq.hoff = (uint32_t)(uintptr_t)(qba_lds_u32 *)hist;
    asm("" : "+v"(wq.hoff));  // held in a VGPR (no instruction is emitted)
    // wave-uniform trip count: pushes and drains always run with the whole wave
    for (uint32_t u = u0;; u += ustride) {
      const bool act = u < nunits;
      if (!__any(act)) break;
      qba_step_l<NP, MODE, SAMP, QPT, false, PK, true, CNT, PW>(u * (4 * QPT), count, first, k0, k1, ps, pat, apat, thr,
                                                            pl, lists, ld, hist, &wq, act);
    }
    while (wq.qn) {  // wave-uniform
      if constexpr (CNT)
        qba_q_drain_pb<NP>(wq, wq.qn < 64 ? wq.qn : 64u);
      else
        qba_q_drain<NP, MODE == 1>(wq, hist, wq.qn < 64 ? wq.qn : 64u);
    }
  } else {
    for (uint32_t u = u0; u < nunits; u += ustride)
      qba_step_l<NP, MODE, SAMP, QPT, false, PK, false, 0, PW>(u * (4 * QPT), count, first, k0, k1, ps, pat, apat,
                                                            thr, pl, lists, ld, hist);
  }
  const uint32_t tid = (wv << 6) | __lane_id();  // == threadIdx.x (above)
  // the remaining < 4 QPT entries: whole quads, then the partial one
  const uint32_t r0 = nunits * (4 * QPT), rq = (count - r0 + 3) >> 2;
  if (bid == nblk - 1 && tid < rq) {
    const uint32_t c0 = r0 + 4 * tid;
    if (c0 + 4 <= count)
      qba_step_l<NP, MODE, SAMP, 1, false, PK, false, CNT, PW>(c0, count, first, k0, k1, ps, pat, apat, thr, pl, lists, ld, hist);
    else
      qba_step_l<NP, MODE, SAMP, 1, true, PK, false, CNT, PW>(c0, count, first, k0, k1, ps, pat, apat, thr, pl, lists, ld, hist);
  }
  if (MODE != 0) {
    __syncthreads();
    uint32_t *row = slab + (size_t)bid * C::NBP;
    bool classic = !CNT;
    if constexpr (CNT) {
      if (qba_pb_flush<NP, BS>(hist, row, (int)tid)) {
        // a pair-bin lane wrapped (never for sampled lists at QBA_PB_BUDGET
        // entries per workgroup): recount this workgroup's entries -- the
        // same units and tail as above -- from the rows it stored, into the
        // classic 32-bit bins (qba_count_quad: exact, order-free)
        __syncthreads();
        for (int i = tid; i < C::NBP; i += BS) hist[i] = 0u;
        __threadfence();  // this workgroup's list stores are complete and visible to its loads
        __syncthreads();
        for (uint32_t u = ((wv * nblk + bid) << 6) | __lane_id(); u < nunits; u += ustride)
          qba_step_l<NP, 2, QBA_S_GENERAL, QPT, false, PK>(u * (4 * QPT), count, first, k0, k1, ps, pat, apat, thr,
                                                         pl, lists, ld, hist);
        if (bid == nblk - 1 && tid < rq) {
          const uint32_t c0 = r0 + 4 * tid;
          if (c0 + 4 <= count)
            qba_step_l<NP, 2, QBA_S_GENERAL, 1, false, PK>(c0, count, first, k0, k1, ps, pat, apat, thr, pl, lists,
                                                         ld, hist);
          else
            qba_step_l<NP, 2, QBA_S_GENERAL, 1, true, PK>(c0, count, first, k0, k1, ps, pat, apat, thr, pl, lists,
                                                        ld, hist);
        }
        __syncthreads();
        if (tid == 0) hist[C::HBL + C::CBL + 1] += 1u;  // stats[1]: recounting workgroups
        classic = true;
      }
    }
    if (classic) {
      uint4 *dst = reinterpret_cast<uint4 *>(row);
      const uint4 *src = reinterpret_cast<const uint4 *>(hist);
      for (int i = tid; i < C::NBP / 4; i += BS) dst[i] = src[i];
    }
    // any point of this kernel precedes the reduction; at the end it leaves
    // the main loop's code placement alone
    if (bid == nblk - 1) qba_zero_outputs<NP>(zero, tid, BS);
  }
}

// CNT 1: pair-bin counting (QbaUsePB kernels only; the launcher picks it for
// launches of at least ctx->pb_min entries).
template <int NP, int MODE, int SAMP, int QPT, int PK, int CNT = 0>
__global__ void QBA_LISTS_BOUNDS
    qba_k_lists(const QbaProgramSet *__restrict__ ps, uint32_t k0, uint32_t k1, uint64_t first,
                uint32_t count, uint8_t *__restrict__ lists, uint64_t ld,
                uint32_t *__restrict__ slab, QbaZero zero) {
  static_assert(!CNT || QbaUsePB<NP, MODE, SAMP, PK>::value, "pair bins: the n = 11 kernels of QbaUsePB only");
  qba_lists_body<NP, MODE, SAMP, QPT, PK, QBA_LBLOCK, CNT>(ps, k0, k1, first, count, lists, ld, slab, zero, 0u);
}

// ---------------------------------------------------------------------------
// Deferred slab reduction (qba_sample_check_deferred / _packed_deferred, qba.h).
// A launch that has few list workgroups (configs[1]: 163 of 512 slots) leaves
// CUs idle, and its separate reduce launch costs a kernel boundary per call.
// A deferred call instead runs the PREVIOUS deferred call's reduction in W
// extra workgroups of its own list kernel (qba_k_lists_def), on two
// alternating slab buffers; qba_flush_deferred reduces the last one
// (qba_k_reduce_def).  Reduce workgroup u owns everything of bin row u:
// H[u][*][*], the pair bins C[u][*] (and, for u = 0, the stats), so it writes
// every output word of u exactly once (plain stores, no atomics, no zeroing
// pass): out = (acc ? out : 0) + the column sum over the slab rows, with the
// derived words (|P_u| = sum_x H[u][0][x] -> P[u], C[u][g][g], H[u][1][u])
// from the same sums.  Bitwise identical to qba_k_reduce's result.
// ---------------------------------------------------------------------------
struct QbaDefer {
  const uint32_t *slab;  // the pending call's slab rows (NBP words apart)
  int rows;              // its list workgroups
  int red;               // reduce workgroups after the list workgroups: W, or 0 (none pending)
  int acc;               // the pending call accumulates into its outputs
  int sacc;              // ... and into the stats (a later chunk of one call)
  int64_t *H, *C, *P, *stats;
};

template <int NP>
__host__ __device__ constexpr int qba_def_cols(int u) {  // slab columns of bin row u
  using C = QCfg<NP>;
  return C::G * C::WP + C::CP + (u == 0 ? C::STATS : 0);
}
// Workgroups per bin row: part 0 owns columns [0, 2 WP) at least (groups 0
// and 1: |P_u| and every word derived from it), the other parts split the rest.
template <int NP>
__host__ __device__ constexpr int qba_def_parts() {
  using C = QCfg<NP>;
  return qba_def_cols<NP>(1) >= 8 * C::WP ? 4 : 1;
}
template <int NP>
__host__ __device__ constexpr int qba_def_wgs() {  // reduce workgroups of one deferred reduction
  return QCfg<NP>::W * qba_def_parts<NP>();
}

// The reduce of part `part` of bin row u by one workgroup of bs threads; sh:
// LDS scratch of (bs + qba_def_cols(0)) words.
template <int NP>
__device__ __forceinline__ void qba_reduce_u(const QbaDefer &d, int u, int part, int tid, int bs, uint32_t *sh) {
  using C = QCfg<NP>;
  typedef unsigned long long u64;
  constexpr int NH = C::G * C::WP, NP4 = qba_def_parts<NP>();
  static_assert(qba_def_cols<NP>(0) <= QBA_DBLOCK && QBA_DBLOCK <= QBA_LBLOCK, "one column per thread at least");
  const int ncu = qba_def_cols<NP>(u);
  constexpr int SPAN = (qba_def_cols<NP>(1) + NP4 - 1) / NP4;
  constexpr int SPAN0 = NP4 == 1 ? qba_def_cols<NP>(0) : (SPAN > 2 * C::WP ? SPAN : 2 * C::WP);
  constexpr int REST = NP4 == 1 ? 1 : (qba_def_cols<NP>(1) - SPAN0 + NP4 - 2) / (NP4 - 1);
  const int c0 = part == 0 ? 0 : SPAN0 + (part - 1) * REST;
  const int c1 = part == 0 ? (SPAN0 < ncu ? SPAN0 : ncu) : (part == NP4 - 1 ? ncu : c0 + REST);
  const int nc = c1 - c0;
  const int S = bs / nc;  // row classes: thread (col, sub) sums rows sub, sub + S, ...
  const int col = c0 + tid % nc, sub = tid / nc;
  if (sub < S) {
    const int w = col < NH ? u * NH + col
                           : col < NH + C::CP ? C::HBL + u * C::CP + (col - NH) : C::HBL + C::CBL + (col - NH - C::CP);
    const uint32_t *src = d.slab + w;
    uint32_t s = 0;
    int r = sub;
    // 16 rows in flight per thread (the rows were written by the previous
    // kernel and come from beyond this XCD's L2)
    for (; r + 15 * S < d.rows; r += 16 * S) {
      uint32_t v[16];
#pragma unroll
      for (int k = 0; k < 16; ++k) v[k] = src[(size_t)(r + k * S) * C::NBP];
#pragma unroll
      for (int k = 0; k < 16; ++k) s += v[k];
    }
    for (; r < d.rows; r += S) s += src[(size_t)r * C::NBP];
    sh[sub * nc + (col - c0)] = s;
  }
  __syncthreads();
  uint32_t *tot = sh + S * nc;  // tot[c - c0]
  if (tid < nc) {
    uint32_t t = 0;
    for (int k = 0; k < S; ++k) t += sh[k * nc + tid];
    tot[tid] = t;  // <= the entries of one launch (< 2^32)
  }
  __syncthreads();
  u64 psz = 0;  // |P_u|: group 0's bins (columns [0, W), part 0)
  if (part == 0) {
#pragma unroll
    for (int x = 0; x < C::W; ++x) psz += tot[x];
  }
  const bool acc = d.acc != 0;
  for (int c = c0 + tid; c < c1; c += bs) {
    if (c < NH) {
      const int g = c / C::WP, x = c - g * C::WP;
      if (x >= C::W) continue;  // row padding
      const u64 v = g == 1 ? (x == u ? psz : 0ull) : (u64)tot[c - c0];  // group 1: part 0 (c < 2 WP)
      int64_t *o = &d.H[(u * C::G + g) * C::W + x];
      *o = (acc ? *o : 0) + (int64_t)v;
    } else if (c < NH + C::CP) {
      int p = c - NH, g = 0;
      while (p >= C::G - 1 - g) p -= C::G - 1 - g++;  // pidx(g, h) inverted
      const int h = g + 1 + p;
      int64_t *o1 = &d.C[(u * C::G + g) * C::G + h], *o2 = &d.C[(u * C::G + h) * C::G + g];
      *o1 = (acc ? *o1 : 0) + (int64_t)tot[c - c0];
      *o2 = (acc ? *o2 : 0) + (int64_t)tot[c - c0];
    } else if (d.stats) {
      int64_t *o = &d.stats[c - NH - C::CP];
      *o = (d.sacc ? *o : 0) + (int64_t)tot[c - c0];
    }
  }
  if (part == 0) {
    for (int g = tid; g < C::G; g += bs) {
      int64_t *o = &d.C[(u * C::G + g) * C::G + g];
      *o = (acc ? *o : 0) + (int64_t)psz;
    }
    if (tid == 0) d.P[u] = (acc ? d.P[u] : 0) + (int64_t)psz;
  }
}

// Sample + check (MODE 1) with the pending deferred call's reduction in the
// LAST d.red workgroups: the list workgroups (slab row = their index) are
// dispatched first, the reduce workgroups into the CUs they leave idle
// (configs[1]: 9.42-9.47 vs 9.68-10.27 us per pass with the reduction ahead,
// profiles/r5/c1)
template <int NP, int SAMP, int QPT, int PK>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, QBA_DBLOCK),
                               amdgpu_waves_per_eu(SAMP == QBA_S_CLOSED ? QBA_DEF_WAVES : 1)))
    qba_k_lists_def(const QbaProgramSet *__restrict__ ps, uint32_t k0, uint32_t k1, uint64_t first,
                    uint32_t count, uint8_t *__restrict__ lists, uint64_t ld, uint32_t *__restrict__ slab,
                    QbaZero zero, QbaDefer d) {
  extern __shared__ __align__(16) uint64_t lds[];
  const uint32_t nl = gridDim.x - (uint32_t)d.red;
  if (blockIdx.x >= nl) {  // workgroup-uniform
    constexpr int NP4 = qba_def_parts<NP>();
    const int r = (int)(blockIdx.x - nl);
    qba_reduce_u<NP>(d, r / NP4, r % NP4, (int)threadIdx.x, QBA_DBLOCK, reinterpret_cast<uint32_t *>(lds));
    return;
  }
  qba_lists_body<NP, 1, SAMP, QPT, PK, QBA_DBLOCK, 0, QBA_DEF_PAIRWISE>(ps, k0, k1, first, count, lists,
                                                                                   ld, slab, zero, 0u, (uint32_t)d.red);
}

// qba_flush_deferred: the last pending reduction on its own.
template <int NP>
__global__ void __launch_bounds__(QBA_LBLOCK) qba_k_reduce_def(QbaDefer d) {
  extern __shared__ __align__(16) uint64_t lds[];
  constexpr int NP4 = qba_def_parts<NP>();
  qba_reduce_u<NP>(d, (int)blockIdx.x / NP4, (int)blockIdx.x % NP4, (int)threadIdx.x, QBA_LBLOCK,
                   reinterpret_cast<uint32_t *>(lds));
}

// The pair-bin kernel with a deferred reduction in its TAIL: the pending
// call's reduce workgroups come after the list workgroups, so they are
// dispatched as list workgroups finish -- into the slots of the ~20 % that
// run one thread-step fewer (1.25e8 entries over 512 x 1024 threads is 29.8
// steps) -- instead of a separate reduce launch after the list kernel.
template <int NP, int QPT, int PK>
__global__ void QBA_LISTS_BOUNDS_PB
    qba_k_lists_pbdef(const QbaProgramSet *__restrict__ ps, uint32_t k0, uint32_t k1, uint64_t first,
                      uint32_t count, uint8_t *__restrict__ lists, uint64_t ld, uint32_t *__restrict__ slab,
                      QbaZero zero, QbaDefer d) {
  extern __shared__ __align__(16) uint64_t lds[];
  const uint32_t nl = gridDim.x - (uint32_t)d.red;
  if (blockIdx.x >= nl) {  // workgroup-uniform
    constexpr int NP4 = qba_def_parts<NP>();
    const int r = (int)(blockIdx.x - nl);
    qba_reduce_u<NP>(d, r / NP4, r % NP4, (int)threadIdx.x, QBA_LBLOCK, reinterpret_cast<uint32_t *>(lds));
    return;
  }
  qba_lists_body<NP, 1, QBA_S_CLOSED, QPT, PK, QBA_LBLOCK, 1>(ps, k0, k1, first, count, lists, ld, slab, zero, 0u,
                                                              (uint32_t)d.red);
}

// Batched independent instances (BASELINE configs[3]): instance i is its own
// run with Philox key seed_base + i over entries [0, count).  A workgroup
// owns whole instances, so its LDS histogram IS the instance's final count
// and is written out directly (no slab, no reduce launch).
// Compiled for 8 waves per SIMD on the closed sampler (configs[3]: 0.743 ->
// 0.728 ms/step, profiles/r5/batched; 53 VGPRs once the per-instance output
// addresses are no longer hoisted across the main loop)
template <int NP, int SAMP, int QPT, int PK>
__global__ void __attribute__((amdgpu_flat_work_group_size(1, QBA_BLOCK),
                               amdgpu_waves_per_eu(SAMP == QBA_S_CLOSED ? 8 : 1)))
    qba_k_batched(const QbaProgramSet *__restrict__ ps, uint64_t seed_base, int64_t n_inst,
                  uint64_t count, uint8_t *__restrict__ lists, uint64_t ld, uint64_t inst_stride,
                  int64_t *__restrict__ H, int64_t *__restrict__ Cc, int64_t *__restrict__ P) {
  using C = QCfg<NP>;
  extern __shared__ __align__(16) uint64_t lds[];
  const uint64_t *pat, *apat, *thr;
  const uint32_t *pl;
  uint32_t *hist = qba_stage<NP, 1, SAMP, QBA_BLOCK>(ps, lds, pat, apat, thr, pl);
  const uint32_t wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  for (int64_t inst = blockIdx.x; inst < n_inst; inst += gridDim.x) {
    for (int i = (int)((wv << 6) | __lane_id()); i < C::NBINS; i += QBA_BLOCK) hist[i] = 0u;
    __syncthreads();
    const uint64_t key = seed_base + (uint64_t)inst;
    const uint32_t k0 = (uint32_t)key, k1 = (uint32_t)(key >> 32);
    uint8_t *L = lists + (uint64_t)inst * inst_stride;
    // QPT quads per thread-step, Q entries counted 64 at a time from the
    // per-wave LDS queue (as qba_k_lists), then the < 4 QPT remaining entries
    const uint32_t nunits = (uint32_t)count / (4 * QPT);
    QbaWaveQ wq;
    wq.base = qba_queue_base<NP>(hist) + wv * (CF<NP>::ND * QBA_QCAP * 4);
    wq.tail = 0;
    wq.qn = 0;
    wq.hoff = (uint32_t)(uintptr_t)(qba_lds_u32 *)hist;
    asm("" : "+v"(wq.hoff));
    for (uint32_t u = (wv << 6) | __lane_id();; u += QBA_BLOCK) {  // wave-uniform trip count
      const bool act = u < nunits;
      if (!__any(act)) break;
      qba_step_l<NP, 1, SAMP, QPT, false, PK, true>(u * (4 * QPT), (uint32_t)count, 0, k0, k1, ps, pat, apat, thr, pl,
                                              L, ld, hist, &wq, act);
    }
    while (wq.qn) qba_q_drain<NP, true>(wq, hist, wq.qn < 64 ? wq.qn : 64u);  // wave-uniform
    // the thread index rebuilt (as in qba_lists_body): nothing derived from
    // threadIdx.x stays live across the main loop to be spilled
    int tid = (int)((wv << 6) | __lane_id());
    asm volatile("" : "+v"(tid));  // opaque: the addresses built from it are not hoisted out of the instance loop
    const uint32_t r0 = nunits * (4 * QPT), rq = ((uint32_t)count - r0 + 3) >> 2;
    if ((uint32_t)tid < rq) {
      const uint32_t c0 = r0 + 4 * (uint32_t)tid;
      if (c0 + 4 <= (uint32_t)count)
        qba_step_l<NP, 1, SAMP, 1, false, PK>(c0, (uint32_t)count, 0, k0, k1, ps, pat, apat, thr, pl, L, ld, hist);
      else
        qba_step_l<NP, 1, SAMP, 1, true, PK>(c0, (uint32_t)count, 0, k0, k1, ps, pat, apat, thr, pl, L, ld, hist);
    }
    __syncthreads();
    int64_t *h = H + inst * C::HB, *c = Cc + inst * C::CB, *p = P + inst * C::W;
    for (int i = tid; i < C::HB; i += QBA_BLOCK) h[i] = qba_hval<NP>(hist, i);
    for (int r = tid; r < C::CB; r += QBA_BLOCK) {
      const int u = r / (C::G * C::G), g = (r / C::G) % C::G, k = r % C::G;
      const int64_t v = g < k ? hist[C::HBL + u * C::CP + C::pidx(g, k)]
                              : g > k ? hist[C::HBL + u * C::CP + C::pidx(k, g)]
                                      : qba_psize<NP>(hist, u);
      c[r] = v;
    }
    for (int u = tid; u < C::W; u += QBA_BLOCK) p[u] = qba_psize<NP>(hist, u);
    __syncthreads();
  }
}

// Slab reduction straight into the int64 outputs (see qba.h for shapes).
// Workgroup (x, y) sums slab rows [y*RP, (y+1)*RP) for 1024 bins (4 per
// thread, 16-B loads) and adds each nonzero partial to the output word(s) the
// bin maps to with integer atomics (order-independent: bitwise
// reproducible): H as counted; a pair bin to C[u][g][h] and C[u][h][g]; group
// 0's bins also to |P_u| -- summed per workgroup in LDS first -- which is P[u],
// every C[u][g][g] and H[u][1][u] (group 1's bins are derived, see
// qba_psize); the stats bins to the stats.  The list kernel of the same
// launch zeroed the outputs unless the call accumulates, so no finalize pass
// or accumulator is needed.
template <int NP>
__global__ void __launch_bounds__(256)
    qba_k_reduce(const uint32_t *__restrict__ slab, int nrows, int64_t *__restrict__ H,
                 int64_t *__restrict__ Cc, int64_t *__restrict__ P, int64_t *__restrict__ stats) {
  using C = QCfg<NP>;
  typedef unsigned long long u64;
  __shared__ u64 psz[C::W];
  if (threadIdx.x < C::W) psz[threadIdx.x] = 0ull;
  __syncthreads();
  const int q = blockIdx.x * 256 + threadIdx.x;  // bin quad
  if (4 * q < C::NBP) {
    const int b0 = blockIdx.y * QBA_RED_ROWS;
    const int b1 = b0 + QBA_RED_ROWS < nrows ? b0 + QBA_RED_ROWS : nrows;
    u64 s[4] = {0ull, 0ull, 0ull, 0ull};
#pragma unroll 8
    for (int b = b0; b < b1; ++b) {
      const uint4 v = reinterpret_cast<const uint4 *>(slab + (size_t)b * C::NBP)[q];
      s[0] += v.x;
      s[1] += v.y;
      s[2] += v.z;
      s[3] += v.w;
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (!s[j]) continue;
      const int b = 4 * q + j;
      if (b < C::HBL) {
        const int u = b / (C::G * C::WP), r = b - u * C::G * C::WP, g = r / C::WP, x = r - g * C::WP;
        if (x >= C::W || g == 1) continue;  // row padding / never counted
        atomicAdd(reinterpret_cast<u64 *>(&H[(u * C::G + g) * C::W + x]), s[j]);
        if (g == 0) atomicAdd(&psz[u], s[j]);
      } else if (b < C::HBL + C::CBL) {
        const int u = (b - C::HBL) / C::CP;
        int p = b - C::HBL - u * C::CP, g = 0;
        while (p >= C::G - 1 - g) p -= C::G - 1 - g++;  // pidx(g, h) inverted
        const int h = g + 1 + p;
        atomicAdd(reinterpret_cast<u64 *>(&Cc[(u * C::G + g) * C::G + h]), s[j]);
        atomicAdd(reinterpret_cast<u64 *>(&Cc[(u * C::G + h) * C::G + g]), s[j]);
      } else if (b < C::NBINS && stats) {
        atomicAdd(reinterpret_cast<u64 *>(&stats[b - C::HBL - C::CBL]), s[j]);
      }
    }
  }
  __syncthreads();
  for (int i = threadIdx.x; i < C::W * (C::G + 2); i += 256) {
    const int u = i / (C::G + 2), k = i - u * (C::G + 2);
    const u64 v = psz[u];
    if (!v) continue;
    int64_t *dst = k < C::G ? &Cc[(u * C::G + k) * C::G + k] : k == C::G ? &P[u] : &H[(u * C::G + 1) * C::W + u];
    atomicAdd(reinterpret_cast<u64 *>(dst), v);
  }
}

// ---------------------------------------------------------------------------
// per-n launchers
// ---------------------------------------------------------------------------

// Persistent grid: every resident workgroup slot of the chip (LDS- and
// register-limited occupancy), fewer when the launch has less work.
static int grid_for(qba_ctx *ctx, const void *kern, size_t lds, uint64_t count, int qpt = QBA_GRID_QPT,
                    int *cap_out = nullptr, int bs = QBA_LBLOCK) {
  // the occupancy query costs tens of microseconds: cached per (kernel, LDS)
  struct Occ {
    const void *k;
    size_t lds;
    int per_cu;
  };
  static thread_local Occ cache[16] = {};
  static thread_local int next = 0;
  int per_cu = 0;
  for (const Occ &o : cache)
    if (o.k == kern && o.lds == lds) per_cu = o.per_cu;
  if (per_cu == 0) {
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, kern, bs, lds) != hipSuccess ||
        per_cu < 1)
      per_cu = 1;
    cache[next] = Occ{kern, lds, per_cu};
    next = (next + 1) % 16;
  }
  const uint64_t nquad = (count + 3) >> 2;
  // >= 2 quads (one wide thread-step) per thread: a small launch (configs[1],
  // 1e6 entries) spreads over 163 workgroups instead of 82
  uint64_t g = (nquad + (uint64_t)qpt * bs - 1) / ((uint64_t)qpt * bs);
  const uint64_t cap = (uint64_t)ctx->num_cus * (uint64_t)per_cu;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  if (cap_out) *cap_out = (int)cap;
  return (int)g;
}

// qba_flush_deferred / qba_flush_pending: the pending call's reduction alone.
template <int NP>
static int qba_flush_def(qba_ctx *ctx) {
  const auto &p = ctx->pend;
  const QbaDefer d{p.slab, p.rows, 0, p.acc, p.sacc, p.H, p.C, p.P, p.stats};
  const size_t lds = (size_t)(QBA_LBLOCK + qba_def_cols<NP>(0)) * sizeof(uint32_t);
  hipLaunchKernelGGL(qba_k_reduce_def<NP>, dim3(qba_def_wgs<NP>()), dim3(QBA_LBLOCK), lds, p.stream, d);
  QBA_HIP(hipGetLastError());
  return QBA_OK;
}

// Sampler of the compiled pair: closed form when proven (n <= 11), else the
// canonical-table fast path, else the general alias-table path.
template <int NP>
static int sampler_of(const QbaProgramSet *hs) {
  if (NP <= QBA_CLOSED_MAX_N && hs->closed) return QBA_S_CLOSED;
  return hs->canonical ? QBA_S_FAST : QBA_S_GENERAL;
}

// LDS bytes of the staged tables for a sampling launch
template <int NP>
static size_t table_lds(const QbaProgramSet *hs, int samp) {
  if (samp == QBA_S_CLOSED) return (size_t)((CF<NP>::WORDS + 3) & ~3) * sizeof(uint32_t);
  return (size_t)(((hs->any_nonuniform ? 3 : 1) * hs->table_total + 1) & ~1) * sizeof(uint64_t);
}

template <int NP>
static int check_closed(const QbaProgramSet *hs) {
  if (hs->closed && (hs->ra != CF<NP>::RA || hs->rb != CF<NP>::RB || hs->rc != CF<NP>::RC ||
                     hs->perm_words != CF<NP>::WORDS || hs->t32 != CF<NP>::T32 ||
                     hs->perm_off != (int32_t)QBA_PERM_OFF))
    return qba_fail(QBA_EINVAL, "closed-form program does not match the kernel's stage layout");
  return QBA_OK;
}

template <int NP>
int qba_launch_lists(qba_ctx *ctx, const QbaLaunch &L) {
  using C = QCfg<NP>;
  const QbaProgramSet *hs = reinterpret_cast<const QbaProgramSet *>(ctx->prog_host[NP]);
  int samp = QBA_S_GENERAL;
  size_t lds = 0;
  if (L.mode != 2) {
    samp = sampler_of<NP>(hs);
    if (int rc = check_closed<NP>(hs)) return rc;
    lds += table_lds<NP>(hs, samp);
  }
  // the fused closed-form kernel and the check of nibble rows count with
  // pair bins (QbaPB, n = 11) when the launch is large enough to repay their
  // flush (a fixed ~2 us per launch: 1e6 entries 17.7 vs 15.0 us, 1.25e8
  // entries 298 vs 313 us, profiles/r4/small_launch); the tests' list_grid
  // knob (qba_test_set_knobs) forces them
  const bool pb = ((L.mode == 1 && QbaUsePB<NP, 1, QBA_S_CLOSED, 0>::value && samp == QBA_S_CLOSED) ||
                   (L.mode == 2 && QbaUsePB<NP, 2, QBA_S_GENERAL, 1>::value && L.packed)) &&
                  (L.count >= ctx->pb_min || ctx->list_grid > 0);
  if (pb) {
    lds += 1024 + (size_t)QbaPB::AREA * sizeof(uint32_t) + (size_t)(QBA_LBLOCK / 64 + 1) * QBA_QCAP * QbaPB::QSLOT;
  } else if (L.mode != 0) {
    lds += (size_t)((C::NBP + 3) & ~3) * sizeof(uint32_t);
    lds += (size_t)(QBA_LBLOCK / 64) * CF<NP>::ND * QBA_QCAP * sizeof(uint32_t) + QBA_QCAP * 4;
  }
  lds = (lds + 15) & ~(size_t)15;
  if (lds == 0) lds = 16;
  // 4*QPT-byte row vectors (QPT quads per thread-step) when the rows allow it
  constexpr uintptr_t VA = 4 * QBA_WIDE_QPT - 1;  // row vectors need their natural alignment
  // (the one-quad step on twice the workgroups for small launches shortens
  // the list kernel -- 8.8 vs 10.1 us at 1e6 entries -- but its workgroups
  // then share CUs with the deferred reduction's: 11.7 vs 10.3 us per
  // configs[1] step, profiles/r3/r3m, r3n; rejected, tools/exp/rejected)
  // nibble rows: the wide step stores one 4-B word per row (QPT = 2)
  const uintptr_t va = L.packed ? 3 : VA;
  const bool wide = !(reinterpret_cast<uintptr_t>(L.lists) & va) && !(L.ld & va);
#define QBA_K(M, S)                                                                          \
  (L.packed ? (wide ? (const void *)qba_k_lists<NP, M, S, 2, 1> : (const void *)qba_k_lists<NP, M, S, 1, 1>) \
            : (wide ? (const void *)qba_k_lists<NP, M, S, QBA_WIDE_QPT, 0> : (const void *)qba_k_lists<NP, M, S, 1, 0>))
  const void *kern = nullptr;
  if (L.mode == 2) {
    kern = QBA_K(2, QBA_S_GENERAL);
    if constexpr (QbaUsePB<NP, 2, QBA_S_GENERAL, 1>::value)
      if (pb)
        kern = wide ? (const void *)qba_k_lists<NP, 2, QBA_S_GENERAL, 2, 1, 1>
                    : (const void *)qba_k_lists<NP, 2, QBA_S_GENERAL, 1, 1, 1>;
  } else if (samp == QBA_S_CLOSED) {
    if constexpr (NP <= QBA_CLOSED_MAX_N) {
      kern = L.mode == 0 ? QBA_K(0, QBA_S_CLOSED) : QBA_K(1, QBA_S_CLOSED);
      if constexpr (QbaUsePB<NP, 1, QBA_S_CLOSED, 0>::value)
        if (pb)
          kern = L.packed ? (wide ? (const void *)qba_k_lists<NP, 1, QBA_S_CLOSED, 2, 1, 1>
                                  : (const void *)qba_k_lists<NP, 1, QBA_S_CLOSED, 1, 1, 1>)
                          : (wide ? (const void *)qba_k_lists<NP, 1, QBA_S_CLOSED, QBA_WIDE_QPT, 0, 1>
                                  : (const void *)qba_k_lists<NP, 1, QBA_S_CLOSED, 1, 0, 1>);
    } else
      return qba_fail(QBA_EUNSUPPORTED, "closed form beyond n = 11");
  } else if (samp == QBA_S_FAST) {
    kern = L.mode == 0 ? QBA_K(0, QBA_S_FAST) : QBA_K(1, QBA_S_FAST);
  } else {
    kern = L.mode == 0 ? QBA_K(0, QBA_S_GENERAL) : QBA_K(1, QBA_S_GENERAL);
  }
#undef QBA_K
  if (lds > 65536) QBA_HIP(hipFuncSetAttribute(kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds));
  int cap = 0;
  int grid = grid_for(ctx, kern, lds, L.count, wide ? (L.packed ? 2 : QBA_GRID_QPT) : 1, &cap);
  if (ctx->list_grid > 0 && grid > ctx->list_grid) grid = ctx->list_grid;  // tests (qba_test_set_knobs)
  // pair bins: at most QBA_PB_BUDGET entries per workgroup and launch (QbaPB;
  // a grid capped by the tests' list_grid knob -- tests that force wraps --
  // at most 2^23, so group 0's 24-bit total, which counts every entry of the
  // workgroup once, stays exact)
  const uint64_t pb_part = ctx->list_grid ? (uint64_t)grid << QBA_PB_FORCED_LOG2 : (uint64_t)cap * QBA_PB_BUDGET;
  if (pb && L.count > pb_part) {
    // later parts accumulate; part boundaries are multiples of 2^18 entries,
    // so the row alignment and the pair parity of `first` are those of the
    // call; only the last part of a deferred call defers its reduction
    const uint64_t part = pb_part;
    QbaLaunch S = L;
    int rc = QBA_OK;
    for (uint64_t done = 0; !rc && done < L.count; done += S.count) {
      S.count = L.count - done < part ? L.count - done : part;
      S.defer = done + S.count >= L.count ? L.defer : 0;
      S.first = L.first + done;
      S.lists = L.lists + (L.packed ? done >> 1 : done);
      S.accumulate = done ? 1 : L.accumulate;
      S.stats_accumulate = done ? 1 : L.stats_accumulate;
      rc = qba_launch_lists<NP>(ctx, S);
    }
    return rc;
  }
  const uint32_t k0 = (uint32_t)L.seed, k1 = (uint32_t)(L.seed >> 32);
  const QbaProgramSet *ps = L.ps;
  uint64_t first = L.first;
  uint32_t count = (uint32_t)L.count;
  uint8_t *lists = L.lists;
  uint64_t ld = L.ld;
  // Deferred reduction: the list kernel also reduces the pending deferred
  // call (W workgroups after its own) when both fit the chip's resident
  // slots together; otherwise the pending one is flushed and this call is
  // reduced at once (its results are then simply complete earlier).
  const void *kd = nullptr;
  // a large pair-bin launch defers into its own tail (qba_k_lists_pbdef)
  const bool pbd = pb && L.defer && L.mode == 1;
  if constexpr (QbaUsePB<NP, 1, QBA_S_CLOSED, 0>::value)
    if (pbd)
      kd = L.packed ? (wide ? (const void *)qba_k_lists_pbdef<NP, 2, 1> : (const void *)qba_k_lists_pbdef<NP, 1, 1>)
                    : (wide ? (const void *)qba_k_lists_pbdef<NP, QBA_WIDE_QPT, 0>
                            : (const void *)qba_k_lists_pbdef<NP, 1, 0>);
  if (!pbd && L.defer && L.mode == 1) {
#define QBA_KD(S)                                                                                  \
  (L.packed ? (wide ? (const void *)qba_k_lists_def<NP, S, 2, 1> : (const void *)qba_k_lists_def<NP, S, 1, 1>) \
            : (wide ? (const void *)qba_k_lists_def<NP, S, QBA_WIDE_QPT, 0> : (const void *)qba_k_lists_def<NP, S, 1, 0>))
    if (samp == QBA_S_CLOSED) {
      if constexpr (NP <= QBA_CLOSED_MAX_N) kd = QBA_KD(QBA_S_CLOSED);
    } else {
      kd = samp == QBA_S_FAST ? QBA_KD(QBA_S_FAST) : QBA_KD(QBA_S_GENERAL);
    }
#undef QBA_KD
  }
  // the deferred kernel runs QBA_DBLOCK-thread workgroups (small launches:
  // more, shorter workgroups; 9.6 vs 10.5 us per configs[1] pass)
  size_t dlds = 0;
  int dgrid = 0, dcap = 0;
  if (pbd) {  // the list kernel's own launch shape; its LDS covers a reduce workgroup's scratch
    dlds = lds;
    if (dlds < (size_t)(QBA_LBLOCK + qba_def_cols<NP>(0)) * sizeof(uint32_t))
      dlds = (size_t)(QBA_LBLOCK + qba_def_cols<NP>(0)) * sizeof(uint32_t);
    if (dlds > 65536) QBA_HIP(hipFuncSetAttribute(kd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dlds));
    dgrid = grid;
  } else if (kd) {
    dlds = table_lds<NP>(hs, samp) +
           (size_t)((C::NBP + 3) & ~3) * sizeof(uint32_t);
    dlds += (size_t)(QBA_DBLOCK / 64) * CF<NP>::ND * QBA_QCAP * sizeof(uint32_t) + QBA_QCAP * 4;
    const size_t rlds = (size_t)(QBA_DBLOCK + qba_def_cols<NP>(0)) * sizeof(uint32_t);
    if (dlds < rlds) dlds = rlds;
    dlds = (dlds + 15) & ~(size_t)15;
    if (dlds > 65536) QBA_HIP(hipFuncSetAttribute(kd, hipFuncAttributeMaxDynamicSharedMemorySize, (int)dlds));
    dgrid = grid_for(ctx, kd, dlds, L.count, wide ? (L.packed ? 2 : QBA_GRID_QPT) : 1, &dcap, QBA_DBLOCK);
    // a launch that would leave CUs idle spreads its units over one workgroup
    // per CU (wave-major units, qba_lists_body): the LDS work of its counting
    // is what bounds it (configs[1]: 163 -> 256 workgroups)
    if (dgrid < ctx->num_cus && ctx->num_cus + qba_def_wgs<NP>() <= dcap) dgrid = ctx->num_cus;
  }
  if (kd && (pbd || dgrid + qba_def_wgs<NP>() <= dcap)) {
    const int grid = dgrid;
    auto &pd = ctx->pend;
    int rc = QBA_OK;
    // a pending call of another n or on another stream is flushed on its own
    // (qba_flush_pending refuses one recorded in another capture state)
    if (pd.flush && (pd.flush != &qba_flush_def<NP> || pd.stream != L.stream))
      if ((rc = qba_flush_pending(ctx, L.stream))) return rc;
    unsigned long long cid = 0;
    const int cap = qba_capture_of(L.stream, &cid);
    if (pd.flush && (cap != ctx->pend_captured || (cap && cid != ctx->pend_capture_id)))
      return qba_fail(QBA_ESTATE, "a deferred reduction is pending across a graph-capture boundary: call "
                                  "qba_flush_deferred before beginning and before ending a capture");
    if (!pd.flush && (rc = qba_slab_order(ctx, L.stream))) return rc;
    const size_t half_need = ((size_t)grid * C::NBP * sizeof(uint32_t) + 255) & ~(size_t)255;
    if (ctx->slab_bytes < 2 * half_need) {
      if ((rc = qba_flush_pending(ctx, L.stream))) return rc;
      if ((rc = qba_ensure_slab(ctx, 2 * half_need))) return rc;  // synchronises before a reallocation
    }
    const size_t half = (ctx->slab_bytes / 2) & ~(size_t)255;
    const int red = pd.flush ? qba_def_wgs<NP>() : 0;
    const int buf = pd.flush ? pd.buf ^ 1 : 0;
    uint32_t *slab = reinterpret_cast<uint32_t *>(reinterpret_cast<char *>(ctx->slab) + (size_t)buf * half);
    QbaDefer d{pd.slab, pd.rows, red, pd.acc, pd.sacc, pd.H, pd.C, pd.P, pd.stats};
    QbaZero zero{L.H, L.C, L.P, L.stats, 0u};  // the reduction writes every output word itself
    void *args[] = {&ps, (void *)&k0, (void *)&k1, &first, &count, &lists, &ld, &slab, &zero, &d};
    QBA_HIP(hipLaunchKernel(kd, dim3(grid + red), dim3(pbd ? QBA_LBLOCK : QBA_DBLOCK), args, dlds, L.stream));
    QBA_HIP(hipGetLastError());
    pd.flush = &qba_flush_def<NP>;
    pd.slab = slab;
    pd.rows = grid;
    pd.acc = L.accumulate;
    pd.sacc = L.stats_accumulate;
    pd.buf = buf;
    pd.H = L.H;
    pd.C = L.C;
    pd.P = L.P;
    pd.stats = L.stats;
    pd.stream = L.stream;
    ctx->pend_captured = cap;
    ctx->pend_capture_id = cid;
    return qba_slab_done(ctx, L.stream);
  }
  if (L.mode != 0) {
    if (int rc = qba_flush_pending(ctx, L.stream)) return rc;
    if (int rc = qba_slab_order(ctx, L.stream)) return rc;
  }
  uint32_t *slab = nullptr;
  if (L.mode != 0) {
    int rc = qba_ensure_slab(ctx, (size_t)grid * C::NBP * sizeof(uint32_t));
    if (rc) return rc;
    slab = reinterpret_cast<uint32_t *>(ctx->slab);
  }
  QbaZero zero{L.H, L.C, L.P, L.stats,
               (L.mode != 0 && !L.accumulate ? 1u : 0u) | (L.mode != 0 && !L.stats_accumulate ? 2u : 0u)};
  void *args[] = {&ps, (void *)&k0, (void *)&k1, &first, &count, &lists, &ld, &slab, &zero};
  QBA_HIP(hipLaunchKernel(kern, dim3(grid), dim3(QBA_LBLOCK), args, lds, L.stream));
  QBA_HIP(hipGetLastError());
  if (L.mode == 0) return QBA_OK;
  // (qba_k_reduce_def as the synchronous reduce: 6.4 vs 5.5 us at 512 slab
  // rows, profiles/r3/r3p -- the atomic column reduce stays)
  const dim3 rgrid((C::NBP / 4 + 255) / 256, (grid + QBA_RED_ROWS - 1) / QBA_RED_ROWS);
  hipLaunchKernelGGL(qba_k_reduce<NP>, rgrid, dim3(256), 0, L.stream, slab, grid, L.H, L.C, L.P, L.stats);
  QBA_HIP(hipGetLastError());
  return qba_slab_done(ctx, L.stream);
}

template <int NP>
int qba_launch_batched(qba_ctx *ctx, const QbaBatch &B) {
  using C = QCfg<NP>;
  const QbaProgramSet *hs = reinterpret_cast<const QbaProgramSet *>(ctx->prog_host[NP]);
  const int samp = sampler_of<NP>(hs);
  if (int rc = check_closed<NP>(hs)) return rc;
  size_t lds = table_lds<NP>(hs, samp) + (size_t)((C::NBP + 3) & ~3) * sizeof(uint32_t);
  lds += (size_t)(QBA_BLOCK / 64) * CF<NP>::ND * QBA_QCAP * sizeof(uint32_t) + QBA_QCAP * 4;
  lds = (lds + 15) & ~(size_t)15;
  const int64_t cap = (int64_t)ctx->num_cus * 16;
  // 8-B row vectors (two quads per thread-step; 4 B for nibble rows) when
  // every row start allows it
  const uintptr_t VA = B.packed ? 3 : 4 * QBA_WIDE_QPT - 1;
  const bool wide = !(reinterpret_cast<uintptr_t>(B.lists) & VA) && !(B.ld & VA) && !(B.inst_stride & VA);
  const int grid = (int)(B.n_inst < cap ? B.n_inst : cap);
  auto go = [&](auto kern) -> int {
    if (lds > 65536)
      QBA_HIP(hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)lds));
    hipLaunchKernelGGL(kern, dim3(grid), dim3(QBA_BLOCK), lds, B.stream, B.ps, B.seed_base,
                       B.n_inst, B.count, B.lists, B.ld, B.inst_stride, B.H, B.C, B.P);
    QBA_HIP(hipGetLastError());
    return QBA_OK;
  };
#define QBA_B(S)                                                                                   \
  (B.packed ? (wide ? go(qba_k_batched<NP, S, 2, 1>) : go(qba_k_batched<NP, S, 1, 1>))                    \
            : (wide ? go(qba_k_batched<NP, S, QBA_WIDE_QPT, 0>) : go(qba_k_batched<NP, S, 1, 0>)))
  if (samp == QBA_S_CLOSED) {
    if constexpr (NP <= QBA_CLOSED_MAX_N) return QBA_B(QBA_S_CLOSED);
    return qba_fail(QBA_EUNSUPPORTED, "closed form beyond n = 11");
  }
  if (samp == QBA_S_FAST) return QBA_B(QBA_S_FAST);
  return QBA_B(QBA_S_GENERAL);
#undef QBA_B
}

