// plan_check.cpp -- drives the host-side C++ of libqba under AddressSanitizer
// and UBSan without a GPU (make -C csrc sanitize; tests/test_sanitizers.py).
//
// Covers qba_plan.cpp (gate validation + permutation mask, union-find
// registers, factor merge + Vose alias tables, closed-form classification,
// permutation stage tables, program image) and the error channel of
// qba_ctx.hip, on tfg.py's own circuits (tfg.py:15-40) for n = 1..15 and on
// malformed inputs.  Register supports, which the library computes on the
// device, are supplied from the circuits' known structure (Bell pairs, |+>
// qubits, GHZ registers: SURVEY.md §8(a) A1/A2).  Exit status 0 = all checks
// passed; any sanitizer report aborts the process.
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../qba_plan.h"

static int failures = 0;
#define CHECK(cond, ...)                         \
  do {                                           \
    if (!(cond)) {                               \
      ++failures;                                \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);              \
      fprintf(stderr, "\n");                     \
    }                                            \
  } while (0)

static int nq_of(int n) { return qba_nq(n); }

// tfg.py:15-22 (notQCorrelated) and tfg.py:25-40 (qCorrelated) gate triples
static std::vector<int32_t> notq_gates(int n) {
  const int nq = nq_of(n), N = (n + 1) * nq;
  std::vector<int32_t> g;
  for (int q = nq; q < N; ++q) g.insert(g.end(), {QBA_GATE_H, q, -1});
  for (int j = 0; j < nq; ++j) g.insert(g.end(), {QBA_GATE_X, j, nq + j});
  return g;
}
static std::vector<int32_t> q_gates(int n, const std::vector<int32_t> &perm) {
  const int nq = nq_of(n), N = (n + 1) * nq;
  std::vector<int32_t> g;
  for (int j = 0; j < nq; ++j) g.insert(g.end(), {QBA_GATE_H, j, -1});
  for (int gg = 1; gg <= n; ++gg)
    for (int j = 0; j < nq; ++j)
      if ((perm[gg - 1] >> (nq - 1 - j)) & 1) g.insert(g.end(), {QBA_GATE_X, gg * nq + j, -1});
  for (int q = nq; q < N; ++q) g.insert(g.end(), {QBA_GATE_X, q, q % nq});
  return g;
}

// support of one register of these circuits: H on one qubit + CX fan-out from
// it (or a lone H): the two patterns "all 0" and "all 1" of its qubits
static HostFactor register_support(const std::vector<int> &qubits, int N) {
  HostFactor f;
  uint64_t ones = 0;
  for (int q : qubits) ones |= 1ull << (N - 1 - q);
  f.pat = {0, ones};
  f.prob = {0.5, 0.5};
  return f;
}

static void check_alias(std::mt19937_64 &rng) {
  for (int k = 1; k <= 256; k = k < 8 ? k + 1 : k * 2) {
    std::vector<double> p(k);
    std::uniform_real_distribution<double> u(0.0, 1.0);
    double tot = 0;
    for (int i = 0; i < k; ++i) tot += (p[i] = (i % 5 == 3) ? 0.0 : u(rng));
    if (tot == 0) p[0] = tot = 1;
    std::vector<uint64_t> thr(k);
    std::vector<int32_t> alias(k);
    CHECK(qba_alias_build(p.data(), k, thr.data(), alias.data()) == QBA_OK, "alias k=%d", k);
    std::vector<double> got(k, 0.0);
    for (int i = 0; i < k; ++i) {
      CHECK(thr[i] <= (1ull << 32) && alias[i] >= 0 && alias[i] < k, "alias table range k=%d", k);
      const double keep = thr[i] / 4294967296.0;
      got[i] += keep / k;
      got[alias[i]] += (1.0 - keep) / k;
    }
    for (int i = 0; i < k; ++i) CHECK(fabs(got[i] - p[i] / tot) < 1e-9, "alias k=%d i=%d", k, i);
  }
  uint64_t thr[2];
  int32_t alias[2];
  const double bad1[2] = {-1.0, 2.0}, bad2[2] = {NAN, 1.0}, bad3[2] = {0.0, 0.0};
  CHECK(qba_alias_build(bad1, 2, thr, alias) == QBA_EINVAL, "negative probability accepted");
  CHECK(qba_alias_build(bad2, 2, thr, alias) == QBA_EINVAL, "NaN accepted");
  CHECK(qba_alias_build(bad3, 2, thr, alias) == QBA_EINVAL, "zero sum accepted");
  CHECK(qba_alias_build(nullptr, 2, thr, alias) == QBA_EINVAL, "null accepted");
  CHECK(std::string(qba_last_error()).find("qba_alias_build") != std::string::npos, "error message");
}

static void check_circuits(std::mt19937_64 &rng) {
  for (int n = 1; n <= QBA_MAX_PARTIES; ++n) {
    const int nq = nq_of(n), N = (n + 1) * nq;
    std::vector<int32_t> perm(n);
    for (int i = 0; i < n; ++i) perm[i] = i + 1;
    std::shuffle(perm.begin(), perm.end(), rng);
    QbaHostProgram prog[2];
    for (int kind = 0; kind < 2; ++kind) {
      const std::vector<int32_t> gates = kind ? q_gates(n, perm) : notq_gates(n);
      std::vector<int32_t> kept;
      CHECK(qba_plan_gates(n, kind, gates.data(), (int)gates.size() / 3, kind ? perm.data() : nullptr, kept) ==
                QBA_OK, "plan_gates n=%d kind=%d: %s", n, kind, qba_last_error());
      const auto regs = qba_plan_registers(N, kept);
      if (kind == 0) {  // nq Bell pairs (j, nq+j) and |+> singletons
        CHECK((int)regs.size() == N - nq, "not-Q registers n=%d: %zu", n, regs.size());
      } else {  // nq GHZ registers {g*nq + j}
        CHECK((int)regs.size() == nq, "Q registers n=%d: %zu", n, regs.size());
        for (const auto &r : regs) CHECK((int)r.size() == n + 1, "GHZ register size n=%d", n);
      }
      std::vector<HostFactor> facs;
      for (const auto &r : regs) facs.push_back(register_support(r, N));
      CHECK(qba_plan_program(n, facs, prog[kind]) == QBA_OK, "plan_program n=%d kind=%d", n, kind);
    }
    std::vector<char> img;
    CHECK(qba_plan_image(n, prog[0], prog[1], img) == QBA_OK, "plan_image n=%d: %s", n, qba_last_error());
    const QbaProgramSet *ps = reinterpret_cast<const QbaProgramSet *>(img.data());
    CHECK(ps->canonical == 1, "canonical flag n=%d", n);
    CHECK(ps->closed == (n <= QBA_CLOSED_MAX_N ? 1 : 0), "closed flag n=%d", n);
    if (ps->closed)  // the list kernels stage the tables with 16-B loads of whole 16-B words
      CHECK(ps->perm_off % 16 == 0 && img.size() >= (size_t)ps->perm_off + 16 * (((size_t)ps->perm_words + 3) / 4),
            "stage tables not 16-B aligned / padded n=%d", n);
    CHECK(ps->perm_off == (int32_t)QBA_PERM_OFF && ps->tab_off % 16 == 0 &&
              ps->tab_off >= ps->perm_off + 16 * ((ps->perm_words + 3) / 4) &&
              img.size() == (size_t)ps->tab_off + 24 * (size_t)ps->table_total,
          "image layout n=%d", n);
    // malformed circuits
    std::vector<int32_t> bad = q_gates(n, perm), kept;
    if (n >= 2) {
      std::swap(perm[0], perm[1]);  // mask no longer matches the permutation
      CHECK(qba_plan_gates(n, 1, bad.data(), (int)bad.size() / 3, perm.data(), kept) == QBA_EINVAL,
            "wrong permutation accepted n=%d", n);
    }
    bad[1] = N;  // target out of range
    CHECK(qba_plan_gates(n, 0, bad.data(), (int)bad.size() / 3, nullptr, kept) == QBA_EINVAL,
          "out-of-range target accepted n=%d", n);
    const int32_t hctl[3] = {QBA_GATE_H, 0, 1};
    CHECK(qba_plan_gates(n, 0, hctl, 1, nullptr, kept) == QBA_EINVAL, "controlled H accepted");
  }
  // a non-uniform factor takes the alias path (u word, thresholds < 2^32)
  std::vector<HostFactor> facs(1);
  facs[0].pat = {0, 1, 2};
  facs[0].prob = {0.1, 0.2, 0.7};
  QbaHostProgram hp;
  CHECK(qba_plan_program(3, facs, hp) == QBA_OK, "non-uniform program");
  CHECK(hp.p.any_nonuniform == 1 && hp.p.fac[0].u_word >= 0 && hp.p.table_len == 4, "non-uniform layout");
}

static void check_perm_tables() {
  for (int n = 1; n <= QBA_CLOSED_MAX_N; ++n) {
    int32_t sizes[6];
    CHECK(qba_perm_tables(n, nullptr, 0, sizes) == QBA_OK, "perm sizes n=%d", n);
    std::vector<uint32_t> w(sizes[5]);
    CHECK(qba_perm_tables(n, w.data(), (int32_t)w.size(), sizes) == QBA_OK, "perm tables n=%d", n);
    uint64_t nf = 1;
    for (int i = 2; i <= n; ++i) nf *= (uint64_t)i;
    CHECK((uint64_t)sizes[0] * sizes[1] * sizes[2] == nf, "radices multiply to n! at n=%d", n);
    if (sizes[5] > 0)
      CHECK(qba_perm_tables(n, w.data(), sizes[5] - 1, sizes) == QBA_EINVAL, "short buffer accepted n=%d", n);
  }
  int32_t sizes[6];
  CHECK(qba_perm_tables(12, nullptr, 0, sizes) == QBA_EINVAL, "n=12 accepted");
}

// qba_host.cpp (CPython set order / tuple hash restatement) on random key
// sequences: the order is a permutation of the distinct keys, nothing is
// read or written outside the buffers (ASan), no signed overflow (UBSan);
// bad arguments are refused.  Equality with the live interpreter is checked
// by tests/test_protocol.py.
extern "C" int qba_host_pyset_order(const int64_t *keys, int64_t n, int64_t *order_out, int64_t *n_out);
extern "C" int qba_host_pytuple_hash(const int64_t *vals, int64_t n, int64_t *hash_out);
static void check_host_sets(std::mt19937_64 &rng) {
  for (int trial = 0; trial < 200; ++trial) {
    const int64_t n = (int64_t)(rng() % 80000);
    std::vector<int64_t> keys(n);
    const int64_t span = trial % 4 == 0 ? 16 : trial % 4 == 1 ? 1000000 : trial % 4 == 2 ? (1ll << 62) : 64;
    for (auto &k : keys) k = (int64_t)(rng() % (uint64_t)span) * (trial % 5 == 0 ? -1 : 1);
    if (trial == 7 && n) keys[0] = INT64_MIN;
    std::vector<int64_t> out(n + 1);
    int64_t m = -1;
    CHECK(qba_host_pyset_order(keys.data(), n, out.data(), &m) == 0, "pyset_order rc");
    std::vector<int64_t> a(keys), b(out.begin(), out.begin() + (m < 0 ? 0 : m));
    std::sort(a.begin(), a.end());
    a.erase(std::unique(a.begin(), a.end()), a.end());
    std::sort(b.begin(), b.end());
    CHECK(a == b, "pyset_order is not a permutation of the distinct keys (trial %d)", trial);
    int64_t h = 0;
    CHECK(qba_host_pytuple_hash(keys.data(), n, &h) == 0, "pytuple_hash rc");
  }
  int64_t m = 0, h = 0;
  CHECK(qba_host_pyset_order(nullptr, 3, nullptr, &m) != 0, "pyset_order accepted NULL keys");
  CHECK(qba_host_pyset_order(nullptr, 0, nullptr, &m) == 0 && m == 0, "empty set");
  CHECK(qba_host_pytuple_hash(nullptr, -1, &h) != 0, "pytuple_hash accepted n < 0");
}

int main() {
  std::mt19937_64 rng(20261016);
  check_alias(rng);
  check_circuits(rng);
  check_perm_tables();
  check_host_sets(rng);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("plan_check: all host checks passed (ASan/UBSan build)\n");
  return 0;
}
