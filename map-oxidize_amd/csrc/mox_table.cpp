// Host-side table utilities of libmox.so (no GPU code): the bytewise table
// order of MOX_F_SORT_BYTES (Rust `String` Ord), applied to a
// table fetched from HBM.  The reference's own order is HashMap-random
// (/root/reference/src/main.rs:177-179); this order is the deterministic one
// callers can ask for.
#include "mox_table.h"

#include <algorithm>
#include <atomic>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

namespace mox_host {
namespace {

struct Ent {
  uint64_t k8;  // first 8 word bytes, big-endian, zero padded
  uint64_t i;   // table index
};

int n_threads() {
  unsigned h = std::thread::hardware_concurrency();
  if (const char* s = getenv("OMP_NUM_THREADS")) h = std::min<unsigned>(h ? h : 64, (unsigned)std::max(1, atoi(s)));
  return (int)std::max(1u, std::min(h ? h : 8u, 32u));
}

template <class F>
void parallel(int T, F f) {
  std::vector<std::thread> th;
  for (int t = 1; t < T; t++) th.emplace_back(f, t);
  f(0);
  for (auto& x : th) x.join();
}

}  // namespace

// Sorts the table (counts[n], offs[n+1], bytes) bytewise ascending by word:
// memcmp over the common length, then the shorter word first.  MSD partition
// by the top 16 bits of the big-endian 8-byte prefix into 65,536 buckets, each
// bucket sorted by (prefix, full compare) on T threads, then the table is
// permuted into fresh arrays that replace the old ones in place.
int sort_table_bytes(uint64_t n, uint64_t* counts, uint64_t* offs, uint8_t* bytes) {
  if (n < 2) return 0;
  const int T = n < (1u << 16) ? 1 : n_threads();
  constexpr int NBK = 1 << 16;
  std::vector<Ent> a(n), b(n);
  std::vector<uint64_t> hist((size_t)T * NBK, 0);
  const uint64_t per = (n + T - 1) / T;
  parallel(T, [&](int t) {
    const uint64_t lo = std::min<uint64_t>(n, per * t), hi = std::min<uint64_t>(n, lo + per);
    uint64_t* hh = &hist[(size_t)t * NBK];
    for (uint64_t i = lo; i < hi; i++) {
      const uint64_t len = offs[i + 1] - offs[i];
      uint8_t k[8] = {0, 0, 0, 0, 0, 0, 0, 0};
      memcpy(k, bytes + offs[i], len < 8 ? len : 8);
      uint64_t v = 0;
      for (int j = 0; j < 8; j++) v = (v << 8) | k[j];
      a[i] = Ent{v, i};
      hh[v >> 48]++;
    }
  });
  // bucket starts, then per-thread cursors inside each bucket
  std::vector<uint64_t> start(NBK + 1, 0);
  for (int k = 0; k < NBK; k++) {
    uint64_t s = 0;
    for (int t = 0; t < T; t++) s += hist[(size_t)t * NBK + k];
    start[k + 1] = start[k] + s;
  }
  for (int k = 0; k < NBK; k++) {
    uint64_t c = start[k];
    for (int t = 0; t < T; t++) {
      const uint64_t x = hist[(size_t)t * NBK + k];
      hist[(size_t)t * NBK + k] = c;
      c += x;
    }
  }
  parallel(T, [&](int t) {
    const uint64_t lo = std::min<uint64_t>(n, per * t), hi = std::min<uint64_t>(n, lo + per);
    uint64_t* cur = &hist[(size_t)t * NBK];
    for (uint64_t i = lo; i < hi; i++) b[cur[a[i].k8 >> 48]++] = a[i];
  });
  std::vector<Ent>().swap(a);
  auto less = [&](const Ent& x, const Ent& y) {
    if (x.k8 != y.k8) return x.k8 < y.k8;
    const uint64_t lx = offs[x.i + 1] - offs[x.i], ly = offs[y.i + 1] - offs[y.i];
    const int c = memcmp(bytes + offs[x.i], bytes + offs[y.i], lx < ly ? lx : ly);
    return c != 0 ? c < 0 : lx < ly;
  };
  std::atomic<int> next{0};
  parallel(T, [&](int) {
    for (int k; (k = next.fetch_add(1)) < NBK;)
      if (start[k + 1] - start[k] > 1) std::sort(b.begin() + start[k], b.begin() + start[k + 1], less);
  });
  // permute into fresh arrays: lengths -> offsets by a blocked parallel scan
  std::vector<uint64_t> nc(n), no(n + 1), part(T + 1, 0);
  parallel(T, [&](int t) {
    const uint64_t lo = std::min<uint64_t>(n, per * t), hi = std::min<uint64_t>(n, lo + per);
    uint64_t s = 0;
    for (uint64_t j = lo; j < hi; j++) {
      const uint64_t i = b[j].i;
      nc[j] = counts[i];
      no[j] = offs[i + 1] - offs[i];
      s += no[j];
    }
    part[t + 1] = s;
  });
  for (int t = 0; t < T; t++) part[t + 1] += part[t];
  const uint64_t nb = part[T];
  uint8_t* nbytes = (uint8_t*)malloc(nb ? nb : 1);
  if (!nbytes) return -1;
  parallel(T, [&](int t) {
    const uint64_t lo = std::min<uint64_t>(n, per * t), hi = std::min<uint64_t>(n, lo + per);
    uint64_t o = part[t];
    for (uint64_t j = lo; j < hi; j++) {
      const uint64_t len = no[j], i = b[j].i;
      memcpy(nbytes + o, bytes + offs[i], len);
      no[j] = o;
      o += len;
    }
  });
  no[n] = nb;
  memcpy(counts, nc.data(), n * 8);
  memcpy(offs, no.data(), (n + 1) * 8);
  memcpy(bytes, nbytes, nb);
  free(nbytes);
  return 0;
}

}  // namespace mox_host
