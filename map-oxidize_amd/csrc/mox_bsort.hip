// Device bytewise sort of a result table (MOX_F_SORT_BYTES; an engine group's
// gathered table): the words in Rust String Ord -- bytewise ascending, a
// proper prefix first -- which is the deterministic key order of SURVEY.md
// §8(b).  The reference's own table order is HashMap-random
// (/root/reference/src/main.rs:177-179); this is presentation, not counting.
//
// Records (32 B) = the word's 16-byte window at the current level as four
// big-endian u32 (so numeric order = byte order, zero padded), a length class
// aux = min(bytes left in the window's suffix, 17), the word's table index and
// a run id.  An LSD radix sort over 8-bit digits, least significant first:
// aux, window bytes 15..0, run id bytes 0..3.  Per digit pass: per-tile
// histograms (tile = 8,192 records), one exclusive scan of the digit-major
// tile counts, and a stable scatter (16-element wave match by 8 ballots,
// per-wave digit counts in LDS, 32 ordered rounds per tile).  Digits whose
// value is the same for every record (read from one up-front histogram of all
// 21 digits) are skipped: zero padding and the run id of level 0 cost nothing.
//
// Ties after level 0 are words that share their first 16 bytes and are both
// longer than 16 bytes (aux == 17 on both sides).  Their maximal runs are
// re-sorted on the next 16 bytes (level 1, 2, ...), with the run id as the
// most significant key so runs stay where they are, until no run is left.
// Two words that agree on every compared byte and differ in length are
// ordered by aux (the shorter one is a proper prefix: first).
#include <algorithm>
#include <cstring>

#include "mox_host.h"

namespace {

struct BRec {
  uint4 k;  // big-endian window bytes
  uint32_t aux, idx, run, pad;
};
constexpr int BS_THREADS = 256;
constexpr int BS_ROUNDS = 32;
constexpr int BS_TILE = BS_THREADS * BS_ROUNDS;  // 8,192 records per tile
constexpr int BS_DIGITS = 21;                    // aux, 16 window bytes, 4 run id bytes
constexpr int SCAN_T = 1024, SCAN_PER = 8, SCAN_TILE = SCAN_T * SCAN_PER;

__device__ __forceinline__ uint32_t digit_of(const BRec& r, int d) {
  if (d == 0) return r.aux;
  if (d <= 16) {  // window byte 16 - d (d = 1: byte 15, the least significant)
    const int b = 16 - d;
    const uint32_t w = b < 4 ? r.k.x : b < 8 ? r.k.y : b < 12 ? r.k.z : r.k.w;
    return (w >> (8 * (3 - (b & 3)))) & 0xFFu;
  }
  return (r.run >> (8 * (d - 17))) & 0xFFu;
}

// Window bytes [16 level, 16 level + 16) of word i, big-endian, zero padded.
__device__ __forceinline__ void window(const uint64_t* offs, const uint8_t* bytes, uint64_t i, uint32_t level, BRec& r) {
  const uint64_t o = offs[i], len = offs[i + 1] - o, a = 16ull * level;
  uint32_t w[4] = {0, 0, 0, 0};
  const uint64_t have = len > a ? len - a : 0;
  const uint32_t nb = have < 16 ? (uint32_t)have : 16u;
  for (uint32_t j = 0; j < nb; j++) w[j >> 2] |= (uint32_t)bytes[o + a + j] << (8 * (3 - (j & 3)));
  r.k = make_uint4(w[0], w[1], w[2], w[3]);
  r.aux = have > 16 ? 17u : (uint32_t)have;
}

}  // namespace

extern "C" __global__ __launch_bounds__(256) void k_bs_init(const uint64_t* offs, const uint8_t* bytes, uint64_t n, BRec* out) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    BRec r;
    window(offs, bytes, i, 0, r);
    r.idx = (uint32_t)i;
    r.run = 0;
    r.pad = 0;
    out[i] = r;
  }
}

// Histograms of all BS_DIGITS digits over every record (gh[d * 256 + v]).
extern "C" __global__ __launch_bounds__(256) void k_bs_ghist(const BRec* in, uint64_t n, unsigned long long* gh) {
  __shared__ uint32_t h[BS_DIGITS * 256];
  for (int i = threadIdx.x; i < BS_DIGITS * 256; i += 256) h[i] = 0;
  __syncthreads();
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    const BRec r = in[i];
#pragma unroll
    for (int d = 0; d < BS_DIGITS; d++) atomicAdd(&h[d * 256 + digit_of(r, d)], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < BS_DIGITS * 256; i += 256)
    if (h[i]) atomicAdd(&gh[i], (unsigned long long)h[i]);
}

// Per-tile digit counts, digit-major: bh[v * ntiles + tile].
extern "C" __global__ __launch_bounds__(BS_THREADS) void k_bs_bhist(const BRec* in, uint64_t n, int d, uint64_t* bh, uint64_t ntiles) {
  __shared__ uint32_t h[256];
  h[threadIdx.x] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * BS_TILE;
  for (int r = 0; r < BS_ROUNDS; r++) {
    const uint64_t i = t0 + (uint64_t)r * BS_THREADS + threadIdx.x;
    if (i < n) atomicAdd(&h[digit_of(in[i], d)], 1u);
  }
  __syncthreads();
  bh[(uint64_t)threadIdx.x * ntiles + blockIdx.x] = h[threadIdx.x];
}

// Stable scatter of one tile by digit d: records in input order get
// consecutive positions per digit starting at the tile's scanned offset.
extern "C" __global__ __launch_bounds__(BS_THREADS) void k_bs_scatter(const BRec* in, BRec* out, uint64_t n, int d, const uint64_t* bo,
                                                                      uint64_t ntiles) {
  __shared__ uint32_t wc[BS_THREADS / 64][256];  // this round's per-wave digit counts
  __shared__ uint64_t base[256];                 // next position of each digit
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  base[tid] = bo[(uint64_t)tid * ntiles + blockIdx.x];
  for (int w = 0; w < BS_THREADS / 64; w++) wc[w][tid] = 0;
  __syncthreads();
  const uint64_t t0 = (uint64_t)blockIdx.x * BS_TILE;
  const uint64_t lt = (1ull << lane) - 1ull;
  for (int r = 0; r < BS_ROUNDS; r++) {
    const uint64_t i = t0 + (uint64_t)r * BS_THREADS + tid;
    const bool ok = i < n;
    BRec rec;
    uint32_t v = 0;
    if (ok) {
      rec = in[i];
      v = digit_of(rec, d);
    }
    // lanes of this wave with the same digit: 8 ballots
    uint64_t eq = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t bal = __ballot(((v >> b) & 1u) != 0);
      eq &= ((v >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t rank = (uint32_t)__popcll(eq & lt);
    if (ok && rank == 0) wc[wv][v] = (uint32_t)__popcll(eq);
    __syncthreads();
    // thread t = digit t: wave prefixes, in wave order
    uint32_t pre[BS_THREADS / 64];
    uint32_t run = 0;
#pragma unroll
    for (int w = 0; w < BS_THREADS / 64; w++) { pre[w] = run; run += wc[w][tid]; }
    __syncthreads();
#pragma unroll
    for (int w = 0; w < BS_THREADS / 64; w++) wc[w][tid] = pre[w];
    __syncthreads();
    if (ok) out[base[v] + wc[wv][v] + rank] = rec;
    __syncthreads();
    base[tid] += run;
#pragma unroll
    for (int w = 0; w < BS_THREADS / 64; w++) wc[w][tid] = 0;
    __syncthreads();
  }
}

// Exclusive scan of u64 (three kernels: tile sums, scan of the tile sums in
// one workgroup, tile scans with their offsets).  In place.
__device__ __forceinline__ uint64_t wg_exscan(uint64_t x, uint64_t* ws, uint64_t& tot) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint64_t inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  if (lane == 63) ws[wv] = inc;
  __syncthreads();
  uint64_t pre = 0, t = 0;
  for (int k = 0; k < nw; k++) { if (k < wv) pre += ws[k]; t += ws[k]; }
  __syncthreads();
  tot = t;
  return pre + inc - x;
}
extern "C" __global__ __launch_bounds__(SCAN_T) void k_scan_sums(const uint64_t* a, uint64_t n, uint64_t* sums) {
  __shared__ uint64_t ws[SCAN_T / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t s = 0;
  for (int j = 0; j < SCAN_PER; j++) {
    const uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + j;
    if (i < n) s += a[i];
  }
  uint64_t tot;
  (void)wg_exscan(s, ws, tot);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}
extern "C" __global__ __launch_bounds__(SCAN_T) void k_scan_top(uint64_t* sums, uint64_t nt, uint64_t* total) {
  __shared__ uint64_t ws[SCAN_T / 64];
  uint64_t carry = 0;
  for (uint64_t c = 0; c < nt; c += SCAN_T) {
    const uint64_t i = c + threadIdx.x;
    const uint64_t x = i < nt ? sums[i] : 0;
    uint64_t tot;
    const uint64_t ex = wg_exscan(x, ws, tot);
    if (i < nt) sums[i] = carry + ex;
    carry += tot;
  }
  if (threadIdx.x == 0 && total) *total = carry;
}
extern "C" __global__ __launch_bounds__(SCAN_T) void k_scan_fin(uint64_t* a, uint64_t n, const uint64_t* sums) {
  __shared__ uint64_t ws[SCAN_T / 64];
  const uint64_t b0 = (uint64_t)blockIdx.x * SCAN_TILE;
  uint64_t v[SCAN_PER], s = 0;
  for (int j = 0; j < SCAN_PER; j++) {
    const uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + j;
    v[j] = i < n ? a[i] : 0;
    s += v[j];
  }
  uint64_t tot;
  uint64_t ex = wg_exscan(s, ws, tot) + sums[blockIdx.x];
  for (int j = 0; j < SCAN_PER; j++) {
    const uint64_t i = b0 + (uint64_t)threadIdx.x * SCAN_PER + j;
    if (i < n) a[i] = ex;
    ex += v[j];
  }
}

// Tie runs after a level: sorted records j - 1 and j are tied when they carry
// the same run id and window and both continue past the window (aux 17).
__device__ __forceinline__ bool tied(const BRec& a, const BRec& b) {
  return a.aux == 17 && b.aux == 17 && a.run == b.run && a.k.x == b.k.x && a.k.y == b.k.y && a.k.z == b.k.z && a.k.w == b.k.w;
}
// in[j] = record j belongs to a run of >= 2 tied records; hd[j] = it starts one.
extern "C" __global__ __launch_bounds__(256) void k_bs_ties(const BRec* r, uint64_t n, uint64_t* in, uint64_t* hd) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const BRec b = r[j];
    const bool tp = j > 0 && tied(r[j - 1], b), tn = j + 1 < n && tied(b, r[j + 1]);
    in[j] = (tp || tn) ? 1 : 0;
    hd[j] = (!tp && tn) ? 1 : 0;
  }
}
// After the exclusive scans of in (cpos) and hd (hx): every record in a run
// goes to the subset at its compact index with its next window and the run id
// base + (heads up to and including its run's), and its sorted position.
extern "C" __global__ __launch_bounds__(256) void k_bs_gather_ties(const BRec* r, uint64_t n, const uint64_t* cpos, const uint64_t* hx,
                                                                   uint64_t m, uint32_t run_base, const uint64_t* offs,
                                                                   const uint8_t* bytes, uint32_t level, BRec* sub, uint64_t* pos) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t c = cpos[j], c1 = j + 1 < n ? cpos[j + 1] : m;
    if (c1 == c) continue;  // not in a run
    const BRec b = r[j];
    const bool head = !(j > 0 && tied(r[j - 1], b));
    BRec o;
    window(offs, bytes, b.idx, level, o);
    o.idx = b.idx;
    o.run = run_base + (uint32_t)(hx[j] + (head ? 1 : 0));
    o.pad = 0;
    sub[c] = o;
    pos[c] = j;
  }
}
extern "C" __global__ __launch_bounds__(256) void k_bs_put_ties(const BRec* sub, uint64_t m, const uint64_t* pos, BRec* r) {
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += (uint64_t)gridDim.x * blockDim.x) r[pos[c]] = sub[c];
}
// Output table in sorted order: counts and lengths, then (after the length
// scan) the bytes.
extern "C" __global__ __launch_bounds__(256) void k_bs_out1(const BRec* r, uint64_t n, const uint64_t* counts, const uint64_t* offs,
                                                             uint64_t* ocounts, uint64_t* olen) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = r[j].idx;
    ocounts[j] = counts[i];
    olen[j] = offs[i + 1] - offs[i];
  }
}
extern "C" __global__ __launch_bounds__(256) void k_bs_out2(const BRec* r, uint64_t n, const uint64_t* offs, const uint8_t* bytes,
                                                             const uint64_t* ooffs, uint8_t* obytes) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint32_t i = r[j].idx;
    const uint64_t a = offs[i], len = offs[i + 1] - a, o = ooffs[j];
    for (uint64_t k = 0; k < len; k++) obytes[o + k] = bytes[a + k];
  }
}

namespace mox_host {
namespace {

int grid_for(uint64_t n) { return (int)std::min<uint64_t>(4096, std::max<uint64_t>(1, (n + 255) / 256)); }

// Exclusive scan of a[0, n) in place on stream s; *total (device) = the sum.
int scan_u64(mox_engine* e, uint64_t* a, uint64_t n, uint64_t* d_total) {
  const uint64_t nt = (n + SCAN_TILE - 1) / SCAN_TILE;
  uint64_t* sums = (uint64_t*)e->s_tmp.p;  // bsort_table sizes s_tmp for the largest scan
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_total, 0, 8, e->stream));
    return MOX_OK;
  }
  hipLaunchKernelGGL(k_scan_sums, dim3((uint32_t)nt), dim3(SCAN_T), 0, e->stream, (const uint64_t*)a, n, sums);
  hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(SCAN_T), 0, e->stream, sums, nt, d_total);
  hipLaunchKernelGGL(k_scan_fin, dim3((uint32_t)nt), dim3(SCAN_T), 0, e->stream, a, n, (const uint64_t*)sums);
  HIPCHK(hipGetLastError());
  return MOX_OK;
}

struct BSort {
  BRec *a, *b;          // records, ping-pong
  uint64_t *bh;         // tile digit counts (256 x tiles)
  unsigned long long* gh;  // BS_DIGITS x 256 global histograms (device) ...
  unsigned long long* h_gh;  // ... and their pinned host copy
  uint64_t* total;      // scan totals (device), 2 words
  uint64_t* h_total;    // pinned
};

// LSD radix sort of recs[0, n) (result in s.a) by (run, window, aux).
int radix_sort(mox_engine* e, BSort& s, uint64_t n) {
  if (n < 2) return MOX_OK;
  hipStream_t st = e->stream;
  HIPCHK(hipMemsetAsync(s.gh, 0, BS_DIGITS * 256 * 8, st));
  hipLaunchKernelGGL(k_bs_ghist, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)s.a, n, s.gh);
  HIPCHK(hipMemcpyAsync(s.h_gh, s.gh, BS_DIGITS * 256 * 8, hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  const uint64_t ntiles = (n + BS_TILE - 1) / BS_TILE;
  for (int d = 0; d < BS_DIGITS; d++) {
    bool uniform = false;
    for (int v = 0; v < 256; v++) uniform |= s.h_gh[d * 256 + v] == n;
    if (uniform) continue;  // every record has the same digit: the order stays
    hipLaunchKernelGGL(k_bs_bhist, dim3((uint32_t)ntiles), dim3(BS_THREADS), 0, st, (const BRec*)s.a, n, d, s.bh, ntiles);
    if (int rc = scan_u64(e, s.bh, 256 * ntiles, s.total)) return rc;
    hipLaunchKernelGGL(k_bs_scatter, dim3((uint32_t)ntiles), dim3(BS_THREADS), 0, st, (const BRec*)s.a, s.b, n, d,
                       (const uint64_t*)s.bh, ntiles);
    HIPCHK(hipGetLastError());
    std::swap(s.a, s.b);
  }
  return MOX_OK;
}

}  // namespace

void bsort_free(mox_engine* e) {
  for (DevBuf* b : {&e->s_counts, &e->s_offs, &e->s_bytes, &e->s_tmp}) {
    dfree(b->p);
    b->p = nullptr;
    b->cap = 0;
  }
}

// The engine's result table (e->res) in bytewise order, on its GPU: the
// sorted copy lives in s_counts / s_offs / s_bytes and becomes the result.
int bsort_table(mox_engine* e) {
  HIPCHK(hipSetDevice(e->device));
  auto& r = e->res;
  const uint64_t n = r.n, nb = r.nb;
  if (n < 2) return MOX_OK;
  if (n >= (1ull << 32)) return fail(MOX_EINVAL, "bytewise sort: %llu words (at most 2^32 - 1)", (unsigned long long)n);
  hipStream_t st = e->stream;
  const uint64_t ntiles = (n + BS_TILE - 1) / BS_TILE;
  const uint64_t scan_n = std::max<uint64_t>(256 * ntiles, n);
  // scratch: 2 record arrays | bh | 3 u64 arrays of n (flags, heads, positions) | subset records x 2 | scan sums | gh | totals
  const uint64_t rec = 32 * n, u64n = 8 * n, bhb = 8 * 256 * ntiles, sums = 8 * ((scan_n + SCAN_TILE - 1) / SCAN_TILE + 16);
  const uint64_t need = 4 * rec + 3 * u64n + bhb + BS_DIGITS * 256 * 8 + 64 + 4096;
  int rc;
  if ((rc = grow_dev(e->s_tmp, sums)) || (rc = grow_dev(e->s_counts, 8 * n + 64)) || (rc = grow_dev(e->s_offs, 8 * (n + 1) + 64)) ||
      (rc = grow_dev(e->s_bytes, nb + 64)))
    return rc;
  uint8_t* pool = nullptr;
  if (hipMalloc((void**)&pool, need) != hipSuccess) return fail(MOX_ENOMEM, "bytewise sort: hipMalloc(%llu) failed", (unsigned long long)need);
  uint8_t* q = pool;
  BSort s;
  BRec* A = (BRec*)q; q += rec;
  BRec* B = (BRec*)q; q += rec;
  BRec* S = (BRec*)q; q += rec;
  BRec* S2 = (BRec*)q; q += rec;
  uint64_t* fin = (uint64_t*)q; q += u64n;
  uint64_t* fhd = (uint64_t*)q; q += u64n;
  uint64_t* pos = (uint64_t*)q; q += u64n;
  s.bh = (uint64_t*)q; q += bhb;
  s.gh = (unsigned long long*)q; q += BS_DIGITS * 256 * 8;
  s.total = (uint64_t*)q;
  static thread_local unsigned long long* h_gh = nullptr;  // pinned, per host thread (engine groups sort from one thread)
  static thread_local uint64_t* h_tot = nullptr;
  if (!h_gh) {
    if (hipHostMalloc((void**)&h_gh, BS_DIGITS * 256 * 8 + 64, hipHostMallocDefault) != hipSuccess) h_gh = nullptr;
    if (hipHostMalloc((void**)&h_tot, 64, hipHostMallocDefault) != hipSuccess) h_tot = nullptr;
  }
  auto done = [&](int code) {
    (void)hipStreamSynchronize(st);
    (void)hipFree(pool);
    return code;
  };
  if (!h_gh || !h_tot) return done(fail(MOX_ENOMEM, "bytewise sort: pinned host allocation failed"));
  s.h_gh = h_gh;
  s.h_total = h_tot;
  // level 0: every word by its first 16 bytes and length class
  hipLaunchKernelGGL(k_bs_init, dim3(grid_for(n)), dim3(256), 0, st, r.offs, r.bytes, n, A);
  s.a = A;
  s.b = B;
  if ((rc = radix_sort(e, s, n))) return done(rc);
  BRec* R = s.a;  // sorted (A or B)
  // levels 1, 2, ...: runs of words sharing all compared bytes
  uint32_t run_base = 1;
  for (uint32_t level = 1;; level++) {
    hipLaunchKernelGGL(k_bs_ties, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, fin, fhd);
    if ((rc = scan_u64(e, fin, n, s.total)) || (rc = scan_u64(e, fhd, n, s.total + 1))) return done(rc);
    HIPCHK(hipMemcpyAsync(h_tot, s.total, 16, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    const uint64_t m = h_tot[0], runs = h_tot[1];
    if (m == 0) break;
    if ((uint64_t)run_base + runs >= (1ull << 32)) return done(fail(MOX_EINVAL, "bytewise sort: too many tie runs"));
    hipLaunchKernelGGL(k_bs_gather_ties, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, (const uint64_t*)fin,
                       (const uint64_t*)fhd, m, run_base, r.offs, r.bytes, level, S, pos);
    s.a = S;
    s.b = S2;
    if ((rc = radix_sort(e, s, m))) return done(rc);
    hipLaunchKernelGGL(k_bs_put_ties, dim3(grid_for(m)), dim3(256), 0, st, (const BRec*)s.a, m, (const uint64_t*)pos, R);
    HIPCHK(hipGetLastError());
    run_base += (uint32_t)runs;
  }
  // the sorted table: counts and lengths, offsets by a scan, bytes
  uint64_t* oc = (uint64_t*)e->s_counts.p;
  uint64_t* oo = (uint64_t*)e->s_offs.p;
  hipLaunchKernelGGL(k_bs_out1, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, r.counts, r.offs, oc, oo);
  if ((rc = scan_u64(e, oo, n, oo + n))) return done(rc);
  hipLaunchKernelGGL(k_bs_out2, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, r.offs, r.bytes, (const uint64_t*)oo,
                     (uint8_t*)e->s_bytes.p);
  HIPCHK(hipGetLastError());
  rc = done(MOX_OK);
  r.counts = oc;
  r.offs = oo;
  r.bytes = (const uint8_t*)e->s_bytes.p;
  r.sorted = true;
  return rc;
}

}  // namespace mox_host
