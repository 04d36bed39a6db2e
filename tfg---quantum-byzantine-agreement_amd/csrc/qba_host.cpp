// qba_host.cpp -- host-only support for the exact-order protocol host: the
// set semantics of tfg.py's packets computed natively.
//
// tfg.py rebuilds every received P as a Python set (tfg.py:240: P =
// set(buff)), every party iterates its own P when it builds its tuple
// (tfg.py:189, 291: tuple(Li[j] for j in P)) and re-sends list(P) (tfg.py:
// 209), so each hop can reorder P; a packet's L is a set of tuples (tfg.py:
// 260), iterated when it is re-sent.  Which order a party sees is CPython's
// set iteration order -- the slot order of its open-addressing hash table --
// and it decides which positions Cond3 compares.  Building
// 31 K-element Python sets and converting them back to arrays dominated the
// exact-mode host.  These functions restate CPython
// 3.10's setobject.c (set_add_entry, set_table_resize, set_insert_clean:
// LINEAR_PROBES 9, PERTURB_SHIFT 5, minimum size 8, growth at fill*5 >=
// mask*3 to used*4, or used*2 beyond 50000) and long_hash / tuplehash
// (xxHash-based, 3.8+) for int64 keys, so the host keeps the iteration order
// as an int64 array without materialising the set.  The Python host checks
// the running interpreter is 3.10 before using them (protocol.py); the CPU
// tests compare them with the live interpreter's sets and hashes.
#include <stdint.h>
#include <string.h>

#include <string>
#include <vector>

#include "qba_internal.h"

namespace {

constexpr uint64_t kM61 = (1ull << 61) - 1;  // _PyHASH_MODULUS

// hash(int(x)) for a machine-size int (long_hash): x mod (2^61 - 1) with the
// sign kept, and -1 -> -2
int64_t py_hash_int(int64_t x) {
  int64_t h;
  if (x >= 0) {
    h = (int64_t)((uint64_t)x % kM61);
  } else {
    const uint64_t a = x == INT64_MIN ? (uint64_t)INT64_MAX + 1u : (uint64_t)(-x);
    h = -(int64_t)(a % kM61);
  }
  return h == -1 ? -2 : h;
}

struct Slot {
  int64_t key;
  int64_t hash;
  bool used;
};

constexpr size_t kLinearProbes = 9;
constexpr unsigned kPerturbShift = 5;
constexpr size_t kMinSize = 8;

void insert_clean(std::vector<Slot> &t, size_t mask, int64_t key, int64_t hash) {
  size_t perturb = (size_t)hash;
  size_t i = (size_t)hash & mask;
  for (;;) {
    if (!t[i].used) {
      t[i] = Slot{key, hash, true};
      return;
    }
    if (i + kLinearProbes <= mask) {
      for (size_t j = 1; j <= kLinearProbes; ++j)
        if (!t[i + j].used) {
          t[i + j] = Slot{key, hash, true};
          return;
        }
    }
    perturb >>= kPerturbShift;
    i = (i * 5 + 1 + perturb) & mask;
  }
}

// The protocol's keys are list positions: 0 <= key < 2^61 - 1, where
// hash(key) == key.  The table then holds the keys alone (8 B per slot,
// -1 = empty): the same probe sequence as the general form below.
void insert_clean_nat(std::vector<int64_t> &t, size_t mask, int64_t key) {
  size_t perturb = (size_t)key;
  size_t i = (size_t)key & mask;
  for (;;) {
    if (t[i] < 0) {
      t[i] = key;
      return;
    }
    if (i + kLinearProbes <= mask) {
      for (size_t j = 1; j <= kLinearProbes; ++j)
        if (t[i + j] < 0) {
          t[i + j] = key;
          return;
        }
    }
    perturb >>= kPerturbShift;
    i = (i * 5 + 1 + perturb) & mask;
  }
}

int64_t pyset_order_nat(const int64_t *keys, int64_t n, int64_t *order_out) {
  size_t mask = kMinSize - 1, fill = 0;
  std::vector<int64_t> t(kMinSize, -1);
  for (int64_t k = 0; k < n; ++k) {
    const int64_t key = keys[k];
    size_t perturb = (size_t)key;
    size_t i = (size_t)key & mask;
    bool present = false, placed = false;
    while (!placed && !present) {
      size_t probes = (i + kLinearProbes <= mask) ? kLinearProbes : 0;
      for (size_t j = i;; ++j) {
        const int64_t e = t[j];
        if (e < 0) {
          t[j] = key;
          ++fill;
          placed = true;
          break;
        }
        if (e == key) {
          present = true;
          break;
        }
        if (probes-- == 0) break;
      }
      if (placed || present) break;
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
    if (present || fill * 5 < mask * 3) continue;  // no deletions: fill == used
    const size_t minused = fill > 50000 ? fill * 2 : fill * 4;
    size_t newsize = kMinSize;
    while (newsize <= minused) newsize <<= 1;
    std::vector<int64_t> nt(newsize, -1);
    for (const int64_t e : t)
      if (e >= 0) insert_clean_nat(nt, newsize - 1, e);
    t.swap(nt);
    mask = newsize - 1;
  }
  int64_t m = 0;
  for (const int64_t e : t)
    if (e >= 0) order_out[m++] = e;
  return m;
}

}  // namespace

extern "C" int qba_host_pyset_order(const int64_t *keys, int64_t n, int64_t *order_out, int64_t *n_out) {
  if (n < 0 || !n_out || (n > 0 && (!keys || !order_out)))
    return qba_fail(QBA_EINVAL, "qba_host_pyset_order: bad arguments");
  bool natural = true;
  for (int64_t k = 0; k < n && natural; ++k) natural = keys[k] >= 0 && (uint64_t)keys[k] < kM61;
  if (natural) {
    *n_out = pyset_order_nat(keys, n, order_out);
    return QBA_OK;
  }
  size_t mask = kMinSize - 1, fill = 0, used = 0;
  std::vector<Slot> t(kMinSize, Slot{0, 0, false});
  for (int64_t k = 0; k < n; ++k) {
    const int64_t key = keys[k], hash = py_hash_int(key);
    size_t perturb = (size_t)hash;
    size_t i = (size_t)hash & mask;
    bool present = false, placed = false;
    while (!placed && !present) {
      size_t probes = (i + kLinearProbes <= mask) ? kLinearProbes : 0;
      size_t j = i;
      for (;;) {
        Slot &e = t[j];
        if (!e.used) {
          e = Slot{key, hash, true};
          ++fill;
          ++used;
          placed = true;
          break;
        }
        if (e.hash == hash && e.key == key) {
          present = true;
          break;
        }
        if (probes == 0) break;
        --probes;
        ++j;
      }
      if (placed || present) break;
      perturb >>= kPerturbShift;
      i = (i * 5 + 1 + perturb) & mask;
    }
    if (present || fill * 5 < mask * 3) continue;
    const size_t minused = used > 50000 ? used * 2 : used * 4;
    size_t newsize = kMinSize;
    while (newsize <= minused) newsize <<= 1;
    std::vector<Slot> nt(newsize, Slot{0, 0, false});
    for (const Slot &e : t)
      if (e.used) insert_clean(nt, newsize - 1, e.key, e.hash);
    t.swap(nt);
    mask = newsize - 1;
    fill = used;
  }
  int64_t m = 0;
  for (const Slot &e : t)
    if (e.used) order_out[m++] = e.key;
  *n_out = m;
  return QBA_OK;
}

extern "C" int qba_host_pytuple_hash(const int64_t *vals, int64_t n, int64_t *hash_out) {
  if (n < 0 || !hash_out || (n > 0 && !vals)) return qba_fail(QBA_EINVAL, "qba_host_pytuple_hash: bad arguments");
  constexpr uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P5 = 2870177450012600261ull;
  uint64_t acc = P5;
  for (int64_t k = 0; k < n; ++k) {
    acc += (uint64_t)py_hash_int(vals[k]) * P2;
    acc = (acc << 31) | (acc >> 33);
    acc *= P1;
  }
  acc += (uint64_t)n ^ (P5 ^ 3527539ull);
  *hash_out = acc == ~0ull ? 1546275796 : (int64_t)acc;
  return QBA_OK;
}
