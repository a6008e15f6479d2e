// Device bytewise sort of a result table (MOX_F_SORT_BYTES; an engine group's
// gathered table): the words in Rust String Ord -- bytewise ascending, a
// proper prefix first -- which is the deterministic key order of SURVEY.md
// §8(b).  The reference's own table order is HashMap-random
// (/root/reference/src/main.rs:177-179); this is presentation, not counting.
//
// Records (16 B) = {key, run, idx}: key = the word's 7-byte window at the
// current level, big-endian in bits 63..8, and in bits 7..0 a length class
// aux = min(bytes left from the window start, 8) (8 = the word goes on past
// the window); run = the tie run the record belongs to (0 at level 0); idx =
// the word's table index.  Numeric order of (run, key) is String Ord on the
// window: equal window bytes order the shorter remainder first.
//
// Each level is an LSD radix sort over 8-bit digits (key bytes 0..7, then run
// bytes 0..3), one ONESWEEP pass per digit (k_os_pass): a tile of 4,096
// records ranks itself stably (bit-sliced ballot match per wave, per-wave digit
// counters in LDS), publishes its digit counts and finds its global offsets by
// a decoupled look-back over the tiles before it (agent-scope status words),
// stages the tile in LDS in digit order and writes each digit's run with
// consecutive stores.  One up-front kernel histograms every digit; a pass over
// a digit whose value is the same for every record is a copy (the pass reads
// the histogram itself: no host round trip between the histogram and the
// passes).
//
// Ties after a level are words that share the window and both go on past it
// (aux == 8 on both sides).  Their maximal runs are re-sorted by the radix
// passes on the next 7 bytes (level 1, 2, ...), with the run id as the most
// significant key so runs stay where they are, until no run is left.  (Sorting
// short runs in place by one thread each was tried and lost: its dependent
// byte loads made it the slowest kernel of the sort.)  The sorted table's
// bytes leave through an LDS stage as aligned 16-byte stores (k_bs_out2).
#include <algorithm>
#include <cstdlib>
#include <cstring>

#include "mox_host.h"

namespace {

struct __attribute__((aligned(16))) BRec {
  uint64_t key;  // window bytes big-endian in bits 63..8, aux in bits 7..0
  uint32_t run, idx;
};
static_assert(sizeof(BRec) == 16, "BRec is one 16-byte load");
constexpr uint32_t WIN = 7;                      // window bytes per level
constexpr uint32_t AUX_MORE = 8;                 // aux: the word continues past the window
constexpr int OS_THREADS = 256;
#ifndef MOX_OS_ITEMS
#define MOX_OS_ITEMS 16
#endif
constexpr int OS_ITEMS = MOX_OS_ITEMS;           // records per thread
constexpr int OS_TILE = OS_THREADS * OS_ITEMS;   // 4,096 records per tile (16 KiB stage per 1,024)
constexpr int OS_WG_PER_CU = OS_ITEMS <= 8 ? 4 : 2;
constexpr int OS_WAVES = OS_THREADS / 64;
constexpr int OS_DIGITS = 12;                    // key bytes 0..7 (0 = aux), run bytes 0..3
// look-back status word of (tile, digit): flag in bits 63..62, count below
constexpr uint64_t ST_AGG = 1ull << 62, ST_INC = 2ull << 62, ST_VAL = (1ull << 62) - 1;
constexpr uint32_t OS_SPIN_MAX = 1u << 22;       // a look-back that waits longer reports a failure (never expected)
constexpr uint64_t TICK_BYTES = 64;              // k_os_pass tile tickets (OS_DIGITS words), zeroed with the status words
static_assert(OS_DIGITS * 4 <= (int)TICK_BYTES, "one ticket per digit pass");

__device__ __forceinline__ uint32_t digit_of(const BRec& r, int d) {
  if (d < 8) return (uint32_t)(r.key >> (8 * d)) & 0xFFu;
  return (r.run >> (8 * (d - 8))) & 0xFFu;
}

// Window bytes [WIN level, WIN level + WIN) of word i and its length class:
// two aligned 8-byte loads and a funnel shift (the table's byte buffers carry
// 64 bytes of slack past their end: grow_dev callers), not one load per byte.
__device__ __forceinline__ uint64_t window(const uint64_t* offs, const uint8_t* bytes, uint64_t i, uint32_t level) {
  const uint64_t o = offs[i], len = offs[i + 1] - o, a = (uint64_t)WIN * level;
  const uint64_t have = len > a ? len - a : 0;
  const uint32_t nb = have < WIN ? (uint32_t)have : WIN;
  uint64_t k = 0;
  if (nb) {
    const uint64_t p = o + a, base = p & ~7ull;
    const uint32_t sh = (uint32_t)(p & 7u);
    const uint64_t* q = reinterpret_cast<const uint64_t*>(bytes + base);
    const uint64_t lo = q[0], hi = sh + nb > 8 ? q[1] : 0ull;
    const uint64_t le = sh ? (lo >> (8 * sh)) | (hi << (64 - 8 * sh)) : lo;  // bytes p .. p + 7, little-endian
    k = __builtin_bswap64(le & ((1ull << (8 * nb)) - 1ull));                   // nb <= 7: byte j at bits 63 - 8 j
  }
  return k | (have > WIN ? AUX_MORE : (uint32_t)have);
}

template <class T>
__device__ __forceinline__ void st_agent(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class T>
__device__ __forceinline__ T ld_agent(const T* p) { return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }

__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

}  // namespace

// Word i's count, byte offset and length, gathered once by the output kernels
// through the sorted records' idx (one 16-byte read instead of three 8-byte
// ones): offset in the low 40 bits of ol (table bytes < 1 TiB), length in the
// high 24 (words < 16 MiB; a table with a longer word is sorted on the host).
struct BPay {
  uint64_t count;
  uint64_t ol;
};
constexpr uint64_t PAY_OFF_BITS = 40, PAY_LEN_MAX = (1ull << 24) - 1;
__device__ __forceinline__ uint64_t pay_off(const BPay& p) { return p.ol & ((1ull << PAY_OFF_BITS) - 1); }
__device__ __forceinline__ uint64_t pay_len(const BPay& p) { return p.ol >> PAY_OFF_BITS; }
extern "C" __global__ __launch_bounds__(256) void k_bs_init(const uint64_t* offs, const uint8_t* bytes, const uint64_t* counts,
                                                            uint64_t n, BRec* out, BPay* pay, unsigned int* err) {
  for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
    BRec r;
    r.key = window(offs, bytes, i, 0);
    r.run = 0;
    r.idx = (uint32_t)i;
    out[i] = r;
    const uint64_t o = offs[i], len = offs[i + 1] - o;
    if (len > PAY_LEN_MAX) atomicOr(err, 4u);  // (the host sorts such a table)
    pay[i] = BPay{counts[i], o | (len << PAY_OFF_BITS)};
  }
}

// The sort's control words before k_bs_init, one launch instead of a memset
// each: flags (err, 3 words), the digit histograms (gh), the level totals and
// run-id bases (total, 16 words; rbs[0] = 1: level 0's run ids end at 1), the
// pass tickets and look-back status words (tick, nst words).
extern "C" __global__ __launch_bounds__(256) void k_bs_zero(unsigned int* err, unsigned long long* gh, uint64_t* total,
                                                            uint64_t* tick, uint64_t nst) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  if (t < 3) err[t] = 0;
  if (t < OS_DIGITS * 256) gh[t] = 0;
  if (t < 8) total[t] = t == 4 ? 1ull : 0ull;  // total + 4 = rbs (u32): rbs[0] = 1, rbs[1] = 0
  for (uint64_t i = t; i < nst; i += stride) tick[i] = 0;
}

// Histograms of digits 0 .. nd - 1 over every record: GH_BLOCKS blocks, one
// contiguous share of the records each, per-wave LDS histograms (a hot digit
// value contends within one wave only), then one global add per non-zero bin
// and block into gh (zeroed before).
constexpr int GH_BLOCKS = 256;
extern "C" __global__ __launch_bounds__(256) void k_bs_ghist(const BRec* in, uint64_t n, int nd, unsigned long long* gh) {
  __shared__ uint32_t h[4][OS_DIGITS * 256];
  const int t = threadIdx.x, wv = t >> 6;
  for (int i = t; i < 4 * OS_DIGITS * 256; i += 256) (&h[0][0])[i] = 0;
  __syncthreads();
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x, lo = (uint64_t)blockIdx.x * per, hi = lo + per < n ? lo + per : n;
  for (uint64_t i = lo + t; i < hi; i += 256) {
    const BRec r = in[i];
    for (int d = 0; d < nd; d++) atomicAdd(&h[wv][d * 256 + digit_of(r, d)], 1u);
  }
  __syncthreads();
  for (int i = t; i < nd * 256; i += 256) {
    const uint32_t x = h[0][i] + h[1][i] + h[2][i] + h[3][i];
    if (x) atomicAdd(&gh[i], (unsigned long long)x);
  }
}

// Exclusive scans of the global digit histograms: gs[d * 256 + v] = first
// output position of digit value v in the pass over digit d (the host skips
// digits whose value is the same for every record).
extern "C" __global__ __launch_bounds__(256) void k_bs_gscan(const unsigned long long* gh, int nd, uint64_t* gs) {
  __shared__ uint64_t ws[4];
  const int t = threadIdx.x, lane = t & 63, wv = t >> 6;
  for (int d = 0; d < nd; d++) {
    const uint64_t x = gh[d * 256 + t];
    uint64_t inc = x;
    for (int o = 1; o < 64; o <<= 1) {
      const uint64_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    uint64_t pre = 0;
    for (int k = 0; k < wv; k++) pre += ws[k];
    gs[d * 256 + t] = pre + inc - x;
    __syncthreads();
  }
}

// One onesweep pass: records in -> out, stably ordered by digit d.  The tile
// index comes from a ticket (*tick, zero at launch) taken when the workgroup
// starts, not from blockIdx.x: every tile a look-back waits on has then
// already started and publishes without waiting on later tiles, whatever
// order the hardware dispatches workgroups in.  status[tile * 256 + v] is
// zero at launch.
extern "C" __global__ __launch_bounds__(OS_THREADS, OS_WG_PER_CU) void k_os_pass(const BRec* __restrict__ in, BRec* __restrict__ out,
                                                                       uint64_t n, int d, const uint64_t* __restrict__ gs,
                                                                       const unsigned long long* __restrict__ gh,
                                                                       uint64_t* status, unsigned int* err,
                                                                       unsigned int* tick) {
  __shared__ __attribute__((aligned(16))) BRec stage[OS_TILE];
  __shared__ uint32_t wcnt[OS_WAVES][256];  // per-wave digit counters, then per-wave offsets inside the digit
  __shared__ uint32_t lstart[256];          // first tile position of each digit
  __shared__ uint64_t gbase[256];           // first output position of this tile's records of each digit
  __shared__ uint32_t ws[OS_WAVES];
  __shared__ uint32_t s_tile;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (tid == 0) s_tile = atomicAdd(tick, 1u);
  __syncthreads();
  const uint32_t tile = s_tile;
  const uint64_t t0 = (uint64_t)tile * OS_TILE;
  const uint32_t tn = (uint32_t)(n - t0 < (uint64_t)OS_TILE ? n - t0 : (uint64_t)OS_TILE);
  for (int w = 0; w < OS_WAVES; w++) wcnt[w][tid] = 0;
  const unsigned long long ghv = gh[d * 256 + tid];  // (in flight with the records)
  // records of wave wv: tile positions wv * 64 ITEMS + i * 64 + lane (input order = (wv, i, lane))
  BRec rec[OS_ITEMS];
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int i = 0; i < OS_ITEMS; i++) {
    const uint32_t p = (uint32_t)(wv * 64 * OS_ITEMS + i * 64 + lane);
    const u32x4 x = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(in + t0 + (p < tn ? p : 0u)));
    rec[i].key = ((uint64_t)x.y << 32) | x.x;
    rec[i].run = x.z;
    rec[i].idx = x.w;
  }
  // every record has the same digit (the histogram holds n in one bin): the
  // order stays, the pass is a copy (no look-back: every tile takes this branch)
  if (__syncthreads_or(ghv == n)) {
#pragma unroll
    for (int i = 0; i < OS_ITEMS; i++) {
      const uint32_t p = (uint32_t)(wv * 64 * OS_ITEMS + i * 64 + lane);
      if (p < tn) out[t0 + p] = rec[i];
    }
    return;
  }
  // stable rank inside the wave: lanes with the same digit by 8 bit-sliced
  // ballots; the lowest such lane advances the wave's counter for the digit
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t rank[OS_ITEMS];
#pragma unroll
  for (int i = 0; i < OS_ITEMS; i++) {
    const uint32_t p = (uint32_t)(wv * 64 * OS_ITEMS + i * 64 + lane);
    const bool ok = p < tn;
    const uint32_t v = digit_of(rec[i], d);
    uint64_t eq = __ballot(ok);
#pragma unroll
    for (int b = 0; b < 8; b++) {
      const uint64_t bal = __ballot((v >> b) & 1u);
      eq &= ((v >> b) & 1u) ? bal : ~bal;
    }
    const uint32_t before = ok ? wcnt[wv][v] : 0u;
    wave_lds_fence();
    if (ok && (eq & lt) == 0) wcnt[wv][v] = before + (uint32_t)__popcll(eq);
    wave_lds_fence();
    rank[i] = before + (uint32_t)__popcll(eq & lt);
  }
  __syncthreads();
  // thread t = digit t: per-wave offsets, the tile's count, its tile start
  uint32_t cnt = 0;
#pragma unroll
  for (int w = 0; w < OS_WAVES; w++) {
    const uint32_t c = wcnt[w][tid];
    wcnt[w][tid] = cnt;
    cnt += c;
  }
  {
    uint32_t inc = cnt;
    for (int o = 1; o < 64; o <<= 1) {
      const uint32_t y = __shfl_up(inc, o);
      if (lane >= o) inc += y;
    }
    if (lane == 63) ws[wv] = inc;
    __syncthreads();
    uint32_t pre = 0;
    for (int k = 0; k < wv; k++) pre += ws[k];
    lstart[tid] = pre + inc - cnt;
  }
  // decoupled look-back: publish the tile's count, sum the counts of the
  // tiles before it back to the first inclusive prefix, publish that
  uint64_t* st = status + (uint64_t)tile * 256 + tid;
  uint64_t sum = 0;
  if (tile == 0) {
    st_agent(st, ST_INC | cnt);
  } else {
    st_agent(st, ST_AGG | cnt);
    const uint64_t* q = st - 256;
    uint32_t spins = 0;
    for (;;) {
      const uint64_t s = ld_agent(q);
      if (s & ST_INC) { sum += s & ST_VAL; break; }
      if (s & ST_AGG) { sum += s & ST_VAL; q -= 256; continue; }
      if (++spins > OS_SPIN_MAX) { atomicOr(err, 1u); break; }
      __builtin_amdgcn_s_sleep(1);
    }
    st_agent(st, ST_INC | (sum + cnt));
  }
  gbase[tid] = gs[d * 256 + tid] + sum;
  __syncthreads();
  // the tile in digit order in LDS, then each digit's run to its place
#pragma unroll
  for (int i = 0; i < OS_ITEMS; i++) {
    const uint32_t p = (uint32_t)(wv * 64 * OS_ITEMS + i * 64 + lane);
    if (p < tn) {
      const uint32_t v = digit_of(rec[i], d);
      stage[lstart[v] + wcnt[wv][v] + rank[i]] = rec[i];
    }
  }
  __syncthreads();
  for (uint32_t j = tid; j < tn; j += OS_THREADS) {
    const BRec r = stage[j];
    const uint32_t v = digit_of(r, d);
    out[gbase[v] + (j - lstart[v])] = r;
  }
}

// Exclusive scan of u64 in place, without any wait on another workgroup (a
// decoupled look-back over tiles measured 27-50 us per scan of 1.4 M values:
// every status read crosses the XCDs' L2s).  k_scan_tsum: tile sums (coalesced
// reads, SC1_TILE values per tile); [k_scan_top: exclusive scan of the tile
// sums in one workgroup, only for more than SC1_TOP tiles]; k_scan_tile: a
// tile's prefix (the sum of the tile sums before it, reduced by the workgroup
// itself, or the scanned sum), its values scanned through LDS (padded: a
// thread's 16 consecutive values in distinct banks), written back coalesced;
// the last tile writes the total.
constexpr int SC1_T = 256, SC1_PER = 16, SC1_TILE = SC1_T * SC1_PER;
constexpr int SC1_PAD = SC1_PER + 1;   // LDS row of a thread: 16 values + 1 pad
constexpr uint64_t SC1_TOP = 4096;     // tile sums a workgroup reduces itself (16 per thread)
__device__ __forceinline__ uint64_t wave_exscan64(uint64_t x, uint64_t& wave_tot) {
  const int lane = threadIdx.x & 63;
  uint64_t inc = x;
  for (int o = 1; o < 64; o <<= 1) {
    const uint64_t y = __shfl_up(inc, o);
    if (lane >= o) inc += y;
  }
  wave_tot = __shfl(inc, 63);
  return inc - x;
}
// block sum of x (SC1_T threads), every thread gets it
__device__ __forceinline__ uint64_t block_sum64(uint64_t x, uint64_t* ws) {
  uint64_t wt;
  (void)wave_exscan64(x, wt);
  __syncthreads();
  if ((threadIdx.x & 63) == 0) ws[threadIdx.x >> 6] = wt;
  __syncthreads();
  uint64_t t = 0;
#pragma unroll
  for (int k = 0; k < SC1_T / 64; k++) t += ws[k];
  return t;
}
extern "C" __global__ __launch_bounds__(SC1_T) void k_scan_tsum(const uint64_t* a, uint64_t n, uint64_t* sums) {
  __shared__ uint64_t ws[SC1_T / 64];
  const uint64_t t0 = (uint64_t)blockIdx.x * SC1_TILE;
  uint64_t x = 0;
#pragma unroll
  for (int k = 0; k < SC1_PER; k++) {
    const uint64_t i = t0 + (uint64_t)k * SC1_T + threadIdx.x;
    x += i < n ? a[i] : 0ull;
  }
  const uint64_t tot = block_sum64(x, ws);
  if (threadIdx.x == 0) sums[blockIdx.x] = tot;
}
extern "C" __global__ __launch_bounds__(1024) void k_scan_top(uint64_t* sums, uint64_t nt) {
  __shared__ uint64_t ws[16];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint64_t carry = 0;
  for (uint64_t c = 0; c < nt; c += 1024) {
    const uint64_t i = c + threadIdx.x;
    const uint64_t x = i < nt ? sums[i] : 0ull;
    uint64_t wt;
    const uint64_t ex = wave_exscan64(x, wt);
    if (lane == 0) ws[wv] = wt;
    __syncthreads();
    uint64_t pre = 0, tot = 0;
    for (int k = 0; k < 16; k++) { if (k < wv) pre += ws[k]; tot += ws[k]; }
    if (i < nt) sums[i] = carry + pre + ex;
    carry += tot;
    __syncthreads();
  }
}
extern "C" __global__ __launch_bounds__(SC1_T) void k_scan_tile(uint64_t* a, uint64_t n, const uint64_t* sums, int scanned,
                                                                uint64_t* total) {
  __shared__ uint64_t v[SC1_T * SC1_PAD];
  __shared__ uint64_t ws[SC1_T / 64];
  const int t = threadIdx.x, wv = t >> 6;
  const uint64_t tile = blockIdx.x, t0 = tile * SC1_TILE;
  // coalesced: value t0 + k 256 + t goes to LDS row (k 256 + t) / 16
#pragma unroll
  for (int k = 0; k < SC1_PER; k++) {
    const uint32_t e = (uint32_t)(k * SC1_T + t);
    const uint64_t i = t0 + e;
    v[(e >> 4) * SC1_PAD + (e & 15u)] = i < n ? a[i] : 0ull;
  }
  uint64_t pre;
  if (scanned) {
    pre = sums[tile];
  } else {  // the sums of the tiles before this one (at most SC1_TOP)
    uint64_t x = 0;
    for (uint64_t k = t; k < tile; k += SC1_T) x += sums[k];
    pre = block_sum64(x, ws);  // (its barriers also publish v)
  }
  __syncthreads();
  uint64_t x[SC1_PER], sum = 0;
#pragma unroll
  for (int j = 0; j < SC1_PER; j++) {
    x[j] = v[t * SC1_PAD + j];
    sum += x[j];
  }
  uint64_t wtot;
  const uint64_t wex = wave_exscan64(sum, wtot);
  __syncthreads();  // (ws reused)
  if ((t & 63) == 0) ws[wv] = wtot;
  __syncthreads();
  uint64_t wpre = 0, agg = 0;
#pragma unroll
  for (int k = 0; k < SC1_T / 64; k++) {
    if (k < wv) wpre += ws[k];
    agg += ws[k];
  }
  uint64_t run = pre + wpre + wex;
#pragma unroll
  for (int j = 0; j < SC1_PER; j++) {
    v[t * SC1_PAD + j] = run;
    run += x[j];
  }
  __syncthreads();
#pragma unroll
  for (int k = 0; k < SC1_PER; k++) {
    const uint32_t e = (uint32_t)(k * SC1_T + t);
    const uint64_t i = t0 + e;
    if (i < n) a[i] = v[(e >> 4) * SC1_PAD + (e & 15u)];
  }
  if (t == 0 && t0 + SC1_TILE >= n && total) *total = pre + agg;  // the last tile
}

// Tie runs after a level: sorted records j - 1 and j are tied when they carry
// the same run id and window and both continue past the window.
__device__ __forceinline__ bool tied(const BRec& a, const BRec& b) {
  return (a.key & 0xFFu) == AUX_MORE && a.key == b.key && a.run == b.run;
}
// fl[j] = in | hd << 32: in = record j belongs to a run of >= 2 tied records,
// hd = it starts one (one exclusive scan then gives both the subset index and
// the heads before it: in <= 1 per record, so the low half never carries).
extern "C" __global__ __launch_bounds__(256) void k_bs_ties(const BRec* r, uint64_t n, uint64_t* fl) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const BRec b = r[j];
    const bool tp = j > 0 && tied(r[j - 1], b), tn = j + 1 < n && tied(b, r[j + 1]);
    fl[j] = ((tp || tn) ? 1ull : 0ull) | ((!tp && tn) ? (1ull << 32) : 0ull);
  }
}
// After the exclusive scan of fl: every record in a run goes to the subset at
// its compact index with its next window and the run id base + (heads up to
// and including its run's), and its sorted position.  The subset is in sorted
// position order, so each run is a contiguous segment of it.  The subset size
// m and the run count come from the scan's total (*tot: m | runs << 32) and
// the level's first run id from *rb_in, all on the device (no host round trip
// per level); block 0 publishes the next level's first run id and resets the
// long-run list for k_bs_segsort.
extern "C" __global__ __launch_bounds__(256) void k_bs_gather_ties(const BRec* r, uint64_t n, const uint64_t* fx, const uint64_t* tot,
                                                                   const uint32_t* rb_in, uint32_t* rb_out, unsigned int* nlrun,
                                                                   unsigned int* err, const uint64_t* offs, const uint8_t* bytes,
                                                                   uint32_t level, BRec* sub, uint32_t* pos) {
  const uint64_t m = tot[0] & 0xFFFFFFFFull, runs = tot[0] >> 32;
  const uint32_t run_base = *rb_in;
  if (blockIdx.x == 0 && threadIdx.x == 0) {
    if ((uint64_t)run_base + runs >= (1ull << 32)) atomicOr(err, 2u);  // too many tie runs (the host fails the sort)
    *rb_out = (uint32_t)(run_base + runs);
    *nlrun = 0;
  }
  if (m == 0) return;
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const uint64_t f = fx[j], c = f & 0xFFFFFFFFull, c1 = j + 1 < n ? (fx[j + 1] & 0xFFFFFFFFull) : m;
    if (c1 == c) continue;  // not in a run
    const BRec b = r[j];
    const bool head = !(j > 0 && tied(r[j - 1], b));
    BRec o;
    o.key = window(offs, bytes, b.idx, level);
    o.idx = b.idx;
    o.run = run_base + (uint32_t)((f >> 32) + (head ? 1 : 0));
    sub[c] = o;
    pos[c] = (uint32_t)j;  // (tables of < 2^32 words)
  }
}
// The subset's runs sorted by key in LDS: a workgroup loads SEG_CH subset
// records (plus SEG_MAX after them) and sorts the runs whose head lies in its
// SEG_CH.  Every record of such a run ranks itself against the run (records
// with a smaller key, or an equal key at a smaller position: a stable order)
// and is written to its run start + rank: the work of a run of L records is
// spread over its L threads, L compares each (one thread per run doing an
// insertion sort left the other threads idle and ran O(L^2) dependent steps:
// ~35 us per level at C2).  A run longer than SEG_MAX is listed (lrun: its first
// record and length) for k_bs_longsort by its head; one longer than RUN_LMAX,
// or one running past the loaded window beyond the list, sets *longrun, and
// the host then radix-sorts the whole subset instead.  Typical runs are a long
// word's punctuation variants: a few records each.
constexpr int SEG_CH = 2048, SEG_MAX = 64, RUN_LMAX = 4096;
extern "C" __global__ __launch_bounds__(256) void k_bs_segsort(BRec* S, const uint64_t* tot, unsigned int* longrun, uint2* lrun,
                                                               unsigned int* nlrun, unsigned int lrun_cap) {
  __shared__ BRec ls[SEG_CH + SEG_MAX];
  const int t = threadIdx.x;
  const uint64_t m = tot[0] & 0xFFFFFFFFull;  // the subset size (k_bs_gather_ties)
  for (uint64_t c0 = (uint64_t)blockIdx.x * SEG_CH; c0 < m; c0 += (uint64_t)gridDim.x * SEG_CH) {
    const uint32_t nl = (uint32_t)(m - c0 < (uint64_t)(SEG_CH + SEG_MAX) ? m - c0 : (uint64_t)(SEG_CH + SEG_MAX));
    for (uint32_t i = t; i < nl; i += 256) ls[i] = S[c0 + i];
    const uint32_t prev_run = c0 > 0 ? S[c0 - 1].run : 0xFFFFFFFFu;
    __syncthreads();
    const uint32_t nh = nl < (uint32_t)SEG_CH ? nl : (uint32_t)SEG_CH;
    for (uint32_t p = t; p < nl; p += 256) {
      const uint32_t run = ls[p].run;
      // head of p's run inside the window (at most SEG_MAX back for a run this
      // workgroup sorts); a head before the window belongs to the previous chunk
      uint32_t h = p;
      while (h > 0 && p - h <= (uint32_t)SEG_MAX && ls[h - 1].run == run) h--;
      if (p - h > (uint32_t)SEG_MAX) continue;  // a run past SEG_MAX: listed by its head
      if (h == 0 && prev_run == run) continue;   // the previous chunk's run
      if (h >= nh) continue;                     // the next chunk's run
      uint32_t e = p;  // last record of the run inside the window
      while (e + 1 < nl && e - h < (uint32_t)SEG_MAX && ls[e + 1].run == run) e++;
      const bool cut = (e + 1 == nl && c0 + nl < m && S[c0 + nl].run == run) || (e - h >= (uint32_t)SEG_MAX && e + 1 < nl && ls[e + 1].run == run);
      if (cut || e - h + 1 > (uint32_t)SEG_MAX) {  // longer than SEG_MAX (or past the window): its head lists it
        if (p != h) continue;
        uint64_t f = c0 + e + 1;
        while (f < m && f - (c0 + h) <= (uint64_t)RUN_LMAX && S[f].run == run) f++;
        const uint64_t len = f - (c0 + h);
        if (len > (uint64_t)RUN_LMAX) { atomicOr(longrun, 1u); continue; }
        const unsigned int q = atomicAdd(nlrun, 1u);
        if (q < lrun_cap) lrun[q] = make_uint2((uint32_t)(c0 + h), (uint32_t)len); else atomicOr(longrun, 1u);
        continue;
      }
      const uint64_t key = ls[p].key;
      uint32_t rank = 0;
      for (uint32_t k = h; k <= e; k++) {
        const uint64_t kk = ls[k].key;
        rank += (kk < key || (kk == key && k < p)) ? 1u : 0u;
      }
      S[c0 + h + rank] = ls[p];
    }
    __syncthreads();  // ls is reloaded for the next chunk
  }
}
// The listed long runs (SEG_MAX < length <= RUN_LMAX), one workgroup each:
// loaded into LDS, padded to a power of two with ~0 keys, bitonic-sorted by
// key, written back.  (Equal keys are words tied on this window too: their
// order is settled by the next level.)
extern "C" __global__ __launch_bounds__(256) void k_bs_longsort(BRec* S, const uint2* lrun, const unsigned int* nlrun,
                                                                unsigned int lrun_cap) {
  __shared__ BRec ls[RUN_LMAX];
  const unsigned int nr = *nlrun < lrun_cap ? *nlrun : lrun_cap;
  const int t = threadIdx.x;
  for (unsigned int q = blockIdx.x; q < nr; q += gridDim.x) {
    const uint2 lr = lrun[q];
    const uint32_t L = lr.y;
    uint32_t P = 1;
    while (P < L) P <<= 1;
    for (uint32_t i = t; i < P; i += 256) {
      if (i < L) ls[i] = S[lr.x + i];
      else { ls[i].key = ~0ull; ls[i].run = ~0u; ls[i].idx = ~0u; }
    }
    __syncthreads();
    for (uint32_t k = 2; k <= P; k <<= 1)
      for (uint32_t j = k >> 1; j > 0; j >>= 1) {
        for (uint32_t i = t; i < P; i += 256) {
          const uint32_t l = i ^ j;
          if (l > i) {
            const bool asc = (i & k) == 0;
            const BRec a = ls[i], b = ls[l];
            if ((a.key > b.key) == asc) { ls[i] = b; ls[l] = a; }
          }
        }
        __syncthreads();
      }
    for (uint32_t i = t; i < L; i += 256) S[lr.x + i] = ls[i];
    __syncthreads();
  }
}
extern "C" __global__ __launch_bounds__(256) void k_bs_put_ties(const BRec* sub, const uint64_t* tot, const uint32_t* pos, BRec* r) {
  const uint64_t m = tot[0] & 0xFFFFFFFFull;
  for (uint64_t c = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; c < m; c += (uint64_t)gridDim.x * blockDim.x) r[pos[c]] = sub[c];
}
// Output table in sorted order: counts and lengths, then (after the length
// scan) the bytes.
extern "C" __global__ __launch_bounds__(256) void k_bs_out1(const BRec* r, uint64_t n, const BPay* pay, uint64_t* ocounts,
                                                             uint64_t* olen) {
  for (uint64_t j = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; j < n; j += (uint64_t)gridDim.x * blockDim.x) {
    const BPay p = pay[r[j].idx];
    ocounts[j] = p.count;
    olen[j] = pay_len(p);
  }
}
// The words' bytes at their sorted offsets: block b writes the bytes of sorted
// words [256 b, 256 b + 256), which are contiguous in the output.  They are
// assembled in LDS from the 16-byte line below their first byte and leave as
// aligned 16-byte stores; the partial first and last lines (shared with the
// neighbouring blocks) byte by byte.  A word of at most 7 bytes that never
// entered a tie run (run 0) takes its bytes from its level-0 key; longer ones
// from the table with dword loads.  A block whose words exceed the stage
// writes them byte by byte.
constexpr int OUT_STAGE = 16384;
extern "C" __global__ __launch_bounds__(256) void k_bs_out2(const BRec* r, uint64_t n, const BPay* pay, const uint8_t* bytes,
                                                             const uint64_t* ooffs, uint8_t* obytes) {
  __shared__ __attribute__((aligned(16))) uint8_t st[OUT_STAGE];
  const int t = threadIdx.x;
  for (uint64_t j0 = (uint64_t)blockIdx.x * 256; j0 < n; j0 += (uint64_t)gridDim.x * 256) {
    const uint64_t j = j0 + t, jend = j0 + 256 < n ? j0 + 256 : n;
    const uint64_t B0 = ooffs[j0], B1 = ooffs[jend], gbase = B0 & ~15ull;
    BRec rec{};
    uint64_t src = 0, len = 0, dst = 0;
    bool inkey = false;
    if (j < n) {
      rec = r[j];
      dst = ooffs[j];
      const uint32_t aux = (uint32_t)(rec.key & 0xFFu);
      inkey = rec.run == 0 && aux < AUX_MORE;  // the level-0 key holds the whole word
      if (inkey) {
        len = aux;
      } else {
        const BPay p = pay[rec.idx];
        src = pay_off(p);
        len = pay_len(p);
      }
    }
    if (B1 - gbase <= (uint64_t)OUT_STAGE) {
      uint8_t* o = st + (dst - gbase);
      if (inkey) {
        for (uint32_t k = 0; k < (uint32_t)len; k++) o[k] = (uint8_t)(rec.key >> (56 - 8 * k));
      } else if (len) {
        const uint32_t* w4 = reinterpret_cast<const uint32_t*>(bytes + (src & ~3ull));
        const uint32_t sh = (uint32_t)(src & 3u), nd = (sh + (uint32_t)len + 3) >> 2;
        for (uint32_t q = 0; q < nd; q += 4) {  // four dword loads in flight at a time
          uint32_t v[4];
#pragma unroll
          for (int u = 0; u < 4; u++) v[u] = q + u < nd ? w4[q + u] : 0u;
#pragma unroll
          for (int u = 0; u < 4; u++)
#pragma unroll
            for (int bb = 0; bb < 4; bb++) {
              const int64_t k = (int64_t)(4 * (q + u) + bb) - (int64_t)sh;
              if (k >= 0 && (uint64_t)k < len) o[k] = (uint8_t)(v[u] >> (8 * bb));
            }
        }
      }
      __syncthreads();
      const uint64_t a0 = (B0 + 15) & ~15ull, a1 = B1 & ~15ull;  // whole lines [a0, a1)
      if (a0 < a1) {
        for (uint64_t q = a0 + 16ull * t; q < a1; q += 16ull * 256)
          *reinterpret_cast<uint4*>(obytes + q) = *reinterpret_cast<const uint4*>(st + (q - gbase));
        if (t < 16 && B0 + t < a0) obytes[B0 + t] = st[B0 - gbase + t];
        if (t >= 16 && t < 32 && a1 + (t - 16) < B1) obytes[a1 + (t - 16)] = st[a1 - gbase + (t - 16)];
      } else if (t < 32 && B0 + t < B1) {
        obytes[B0 + t] = st[B0 - gbase + t];
      }
      __syncthreads();  // the stage is rewritten by the next step
    } else if (inkey) {
      for (uint32_t k = 0; k < (uint32_t)len; k++) obytes[dst + k] = (uint8_t)(rec.key >> (56 - 8 * k));
    } else {
      for (uint64_t k = 0; k < len; k++) obytes[dst + k] = bytes[src + k];
    }
  }
}

namespace mox_host {
namespace {

int grid_for(uint64_t n) { return (int)std::min<uint64_t>(4096, std::max<uint64_t>(1, (n + 255) / 256)); }

// Exclusive scan of a[0, n) in place on the engine stream (k_scan_tsum,
// [k_scan_top,] k_scan_tile); *d_total (device) = the sum.  sums: scratch of
// scan_sum_words(n) words.
uint64_t scan_sum_words(uint64_t n) { return (n + SC1_TILE - 1) / SC1_TILE + 8; }
int scan_u64(mox_engine* e, uint64_t* a, uint64_t n, uint64_t* d_total, uint64_t* sums) {
  if (n == 0) {
    HIPCHK(hipMemsetAsync(d_total, 0, 8, e->stream));
    return MOX_OK;
  }
  const uint64_t nt = (n + SC1_TILE - 1) / SC1_TILE;
  if (nt > 0x7FFFFFFFull) return fail(MOX_EINVAL, "scan: too many tiles");
  hipLaunchKernelGGL(k_scan_tsum, dim3((uint32_t)nt), dim3(SC1_T), 0, e->stream, (const uint64_t*)a, n, sums);
  const int scanned = nt > SC1_TOP ? 1 : 0;
  if (scanned) hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(1024), 0, e->stream, sums, nt);
  hipLaunchKernelGGL(k_scan_tile, dim3((uint32_t)nt), dim3(SC1_T), 0, e->stream, a, n, (const uint64_t*)sums, scanned, d_total);
  HIPCHK(hipGetLastError());
  return MOX_OK;
}

struct BSort {
  BRec *a, *b;                // records, ping-pong
  unsigned long long* gh;     // OS_DIGITS x 256 global histograms (device)
  uint64_t* gs;               // ... their exclusive scans
  uint64_t* status;           // look-back status words: 256 per tile, one region per digit pass (or one reused region)
  bool one_region;            // one status region, zeroed again before every pass (big tables)
  unsigned int* err;          // look-back timeout flag
  unsigned int* tick;         // OS_DIGITS tile tickets (one per digit pass), just below status
};

// LSD radix sort of s.a[0, n) by its first nd digits (key bytes 0..7, then
// run bytes), one onesweep pass per digit (a copy for a digit that is the same
// for every record); the result ends in s.a.  No host round trip.  zeroed:
// gh, the tickets and the status regions were zeroed by k_bs_zero (the first
// sort of a bsort_once); else (the checked mode's subset sorts) here.
int radix_sort(mox_engine* e, BSort& s, uint64_t n, int nd, bool zeroed) {
  if (n < 2) return MOX_OK;
  hipStream_t st = e->stream;
  const uint64_t ntiles = (n + OS_TILE - 1) / OS_TILE;
  if (ntiles > 0x7FFFFFFFull) return fail(MOX_EINVAL, "bytewise sort: too many tiles");
  // the tile tickets and the status words of every pass (a region per digit; a
  // big table's single region is zeroed again before each later pass)
  const size_t region = (size_t)ntiles * 256 * 8;
  if (!zeroed) {
    HIPCHK(hipMemsetAsync(s.gh, 0, (size_t)nd * 256 * 8, st));
    HIPCHK(hipMemsetAsync(s.tick, 0, TICK_BYTES + (s.one_region ? 1 : (size_t)nd) * region, st));
  }
  hipLaunchKernelGGL(k_bs_ghist, dim3(GH_BLOCKS), dim3(256), 0, st, (const BRec*)s.a, n, nd, s.gh);
  hipLaunchKernelGGL(k_bs_gscan, dim3(1), dim3(256), 0, st, (const unsigned long long*)s.gh, nd, s.gs);
  for (int d = 0; d < nd; d++) {
    if (s.one_region && d) HIPCHK(hipMemsetAsync(s.status, 0, region, st));
    hipLaunchKernelGGL(k_os_pass, dim3((uint32_t)ntiles), dim3(OS_THREADS), 0, st, (const BRec*)s.a, s.b, n, d,
                       (const uint64_t*)s.gs, (const unsigned long long*)s.gh,
                       s.status + (s.one_region ? 0 : (size_t)d * ntiles * 256), s.err, s.tick + d);
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
  if (e->h_bsort) (void)hipHostFree(e->h_bsort);
  e->h_bsort = nullptr;
}

// The engine's result table (e->res) in bytewise order, on its GPU: the
// sorted copy lives in s_counts / s_offs / s_bytes and becomes the result.
// Scratch (s_tmp) is engine-owned and reused across calls: about 60 bytes per
// word (76 in the checked mode, which keeps the tie subset apart) plus the
// look-back status (6 bytes per word, or 0.5 when a table's per-digit regions
// would pass 256 MiB and one region is reused).  When it does not fit next to
// the engine's pass buffers (C4 at 16 GiB: 1.37e9 words, ~84 GB), the big
// record arrays borrow the pass scratch that is dead once a table is built
// (cold regions, split buffers, reduce outputs, weighted records; the table
// itself is never borrowed) and only the rest is allocated.
// One attempt; returns -1 (nothing changed in e->res) when an eager level met
// a tie run the unchecked mode cannot sort: the caller runs it again checked.
int bsort_once(mox_engine* e, bool checked) {
  HIPCHK(hipSetDevice(e->device));
  auto& r = e->res;
  const uint64_t n = r.n, nb = r.nb;
  if (n < 2) return MOX_OK;
  if (n >= (1ull << 32)) return fail(MOX_EINVAL, "bytewise sort: %llu words (at most 2^32 - 1)", (unsigned long long)n);
  // MOX_BSORT_MAX_WORDS: the most words the device sort takes (a bigger table
  // is sorted on the host, as when the sort's scratch does not fit)
  if (const char* cap = getenv("MOX_BSORT_MAX_WORDS"))
    if (n > strtoull(cap, nullptr, 10))
      return fail(MOX_ENOMEM, "bytewise sort: %llu words, MOX_BSORT_MAX_WORDS=%s", (unsigned long long)n, cap);
  // (40-bit word offsets in the payload: a bigger table is sorted on the host, as on MOX_ENOMEM)
  if (nb >> PAY_OFF_BITS) return fail(MOX_ENOMEM, "bytewise sort: %llu table bytes (device sort: < 1 TiB)", (unsigned long long)nb);
  hipStream_t st = e->stream;
  const uint64_t ntiles = (n + OS_TILE - 1) / OS_TILE;
  // scratch: records A, B, subset S, payload | run flags, positions | status | gh, gs | scan sums | totals, err
  // (a table whose per-digit status regions would pass 256 MiB reuses one region)
  const bool one_region = 8ull * OS_DIGITS * 256 * ntiles > (256ull << 20);
  // (every array a multiple of 256 bytes: what follows stays aligned for its 8-byte atomics)
  const uint64_t rec = (16 * n + 255) & ~255ull, u64n = (8 * n + 255) & ~255ull, u32n = (4 * n + 255) & ~255ull;
  const uint64_t sums = 8ull * scan_sum_words(n);
  const uint64_t stb = 8ull * (one_region ? 1 : OS_DIGITS) * 256 * ntiles;
  const unsigned int lrun_cap = (unsigned int)std::min<uint64_t>(1u << 20, n / 4 + 16);  // k_bs_longsort's run list
  const uint64_t small = 8ull * lrun_cap + TICK_BYTES + stb + 2 * OS_DIGITS * 256 * 8 + sums + 256;
  // A, B, S (the tie subset: in the checked mode only; else the radix pass's
  // free ping-pong buffer), pay, fin, pos
  const uint64_t big[6] = {rec, rec, checked ? rec : 0, rec, u64n, u32n};
  uint8_t* bp[6] = {nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
  int rc;
  if ((rc = grow_dev(e->s_counts, 8 * n + 64)) || (rc = grow_dev(e->s_offs, 8 * (n + 1) + 64)) || (rc = grow_dev(e->s_bytes, nb + 64)))
    return rc;
  uint64_t need = small;
  for (uint64_t b : big) need += b;
  rc = grow_dev(e->s_tmp, need);
  if (rc == MOX_ENOMEM) {
    (void)hipGetLastError();  // the failed hipMalloc's error is not a later launch's
    const Work& w = e->w;  // (the table is in t_*, or in the gather / sort buffers: never in these)
    struct Slab { uint8_t* p; uint64_t left; };
    Slab slab[] = {{(uint8_t*)w.cold, w.cold ? (uint64_t)w.map_grid * NB * w.cold_cap * 16 : 0},
                   {(uint8_t*)w.uk, w.uk ? w.uniq_cap * 16 : 0},
                   {(uint8_t*)w.split_k, w.split_k ? w.split_k_cap * 16 : 0},
                   {(uint8_t*)w.uc, w.uc ? w.uniq_cap * 8 : 0},
                   {(uint8_t*)w.w, w.w ? w.w_cap * sizeof(WRec) : 0},
                   {(uint8_t*)w.w_sorted, w.w_sorted ? w.w_cap * sizeof(WRec) : 0},
                   {(uint8_t*)w.ui, w.ui ? w.uniq_cap * 4 : 0}};
    need = small;
    for (int k = 0; k < 6; k++) {
      if (!big[k]) continue;
      for (auto& sl : slab)
        if (sl.p && sl.left >= big[k]) {
          bp[k] = sl.p;
          const uint64_t used = (big[k] + 255) & ~255ull;
          sl.p += used;
          sl.left = sl.left > used ? sl.left - used : 0;
          break;
        }
      if (!bp[k]) need += big[k];
    }
    rc = grow_dev(e->s_tmp, need);
    if (rc) {
      size_t fr = 0, to = 0;
      (void)hipMemGetInfo(&fr, &to);
      (void)hipGetLastError();
      int nbor = 0;
      for (uint8_t* p : bp) nbor += p != nullptr;
      return fail(MOX_ENOMEM, "bytewise sort: %llu words need %llu scratch bytes besides %d borrowed arrays; %zu of %zu bytes free",
                  (unsigned long long)n, (unsigned long long)need, nbor, fr, to);
    }
  }
  if (rc) return rc;
  if (!e->h_bsort) HIPCHK(hipHostMalloc((void**)&e->h_bsort, OS_DIGITS * 256 * 8 + 64, hipHostMallocDefault));
  uint8_t* q = (uint8_t*)e->s_tmp.p;
  for (int k = 0; k < 6; k++)
    if (!bp[k] && big[k]) { bp[k] = q; q += big[k]; }
  BRec* A = (BRec*)bp[0];
  BRec* B = (BRec*)bp[1];
  BRec* S = (BRec*)bp[2];  // (nullptr unless checked: then the free ping-pong buffer below)
  BPay* pay = (BPay*)bp[3];
  uint64_t* fin = (uint64_t*)bp[4];
  uint32_t* pos = (uint32_t*)bp[5];
  uint2* lrun = (uint2*)q; q += 8ull * lrun_cap;
  BSort s;
  s.tick = (unsigned int*)q; q += TICK_BYTES;
  s.status = (uint64_t*)q; q += stb;
  s.one_region = one_region;
  s.gh = (unsigned long long*)q; q += OS_DIGITS * 256 * 8;
  s.gs = (uint64_t*)q; q += OS_DIGITS * 256 * 8;
  uint64_t* ssum = (uint64_t*)q; q += sums;
  uint64_t* total = (uint64_t*)q; q += 64;  // [0] subset size [1] runs
  s.err = (unsigned int*)q;
  uint64_t* h_tot = (uint64_t*)(e->h_bsort + OS_DIGITS * 256);
  // err: [0] look-back timeout [1] radix fallback [2] long runs (k_bs_segsort); gh; total / rbs; tickets + status
  {
    const uint64_t nst = (TICK_BYTES + (one_region ? 1 : 8) * (uint64_t)ntiles * 256 * 8) / 8;  // level 0: 8 digits
    hipLaunchKernelGGL(k_bs_zero, dim3((uint32_t)std::min<uint64_t>(4096, std::max<uint64_t>(16, (nst + 255) / 256))), dim3(256), 0,
                       st, s.err, s.gh, total, (uint64_t*)s.tick, nst);
  }
  // level 0: every word by its first 7 bytes and length class
  hipLaunchKernelGGL(k_bs_init, dim3(grid_for(n)), dim3(256), 0, st, r.offs, r.bytes, r.counts, n, A, pay, s.err);
  s.a = A;
  s.b = B;
  if ((rc = radix_sort(e, s, n, 8, true))) return rc;
  BRec* R = s.a;                 // sorted (A or B)
  BRec* S2 = R == A ? B : A;     // the other one is free: the subset's ping-pong partner (checked), or the subset
  if (!checked) S = S2;
  // levels 1, 2, ...: runs of words sharing every compared byte, re-sorted on
  // the next window (by run: short runs in LDS by k_bs_segsort, runs of up to
  // RUN_LMAX by k_bs_longsort).  The first EAGER_LEVELS levels (words up to 21
  // bytes) run with no host round trip: their kernels take the subset size and
  // run ids from the device.  Then one read-back: the subset size of the next
  // level and the flags.  Further levels (longer words tied on 21 bytes) read
  // their subset size back one level at a time.  A run past RUN_LMAX (or past
  // the long-run list) makes the whole sort run again in the checked mode, where
  // every level reads back and such a subset is radix-sorted with the run id as
  // the most significant digits (never seen on the benchmark corpora).
  constexpr uint32_t EAGER_LEVELS = 2;
  unsigned int* longrun = s.err + 1;  // [0] a run past RUN_LMAX or the list  [1] listed long runs
  uint64_t* lvt = total;                                // lvt[level % 4]: the level's scan total (m | runs << 32)
  uint32_t* rbs = (uint32_t*)(total + 4);               // rbs[level % 4]: the level's first run id
  uint32_t run_base = 1;  // checked mode only (rbs[0] = 1: k_bs_zero)
  uint64_t* oc = (uint64_t*)e->s_counts.p;
  uint64_t* oo = (uint64_t*)e->s_offs.p;
  // the sorted table: counts and lengths, offsets by a scan, bytes
  auto output = [&]() -> int {
    hipLaunchKernelGGL(k_bs_out1, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, (const BPay*)pay, oc, oo);
    if (int rc2 = scan_u64(e, oo, n, oo + n, ssum)) return rc2;
    hipLaunchKernelGGL(k_bs_out2, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, (const BPay*)pay, r.bytes,
                       (const uint64_t*)oo, (uint8_t*)e->s_bytes.p);
    HIPCHK(hipGetLastError());
    return MOX_OK;
  };
  bool out_done = false;  // the output kernels ran after the last level
  for (uint32_t level = 1;; level++) {
    uint64_t* lt = lvt + (level & 3);
    hipLaunchKernelGGL(k_bs_ties, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, fin);
    if ((rc = scan_u64(e, fin, n, lt, ssum))) return rc;
    uint64_t m = n, runs = 0;
    if (checked || level > EAGER_LEVELS) {
      // the first level that reads its size back usually finds no tie left (no
      // word tied on 21 bytes): the output kernels go first, on speculation, so
      // that the one read-back also completes the sort (redone after the last
      // level otherwise)
      const bool spec = !checked && level == EAGER_LEVELS + 1;
      if (spec && (rc = output())) return rc;
      HIPCHK(hipMemcpyAsync(h_tot, lt, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipMemcpyAsync(h_tot + 2, s.err, 8, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      const uint32_t fl0 = (uint32_t)h_tot[2], fl1 = (uint32_t)(h_tot[2] >> 32);
      if (fl0 & 1u) return fail(MOX_EHIP, "bytewise sort: a look-back wait timed out");
      if (fl0 & 2u) return fail(MOX_EINVAL, "bytewise sort: too many tie runs");
      if (fl0 & 4u) return fail(MOX_ENOMEM, "bytewise sort: a word of 16 MiB or more (sorted on the host)");
      if (fl1 && !checked) return -1;  // a long run in an eager level: run again, checked
      m = h_tot[0] & 0xFFFFFFFFull;
      runs = h_tot[0] >> 32;
      if (m == 0) {
        out_done = spec;
        break;
      }
    }
    hipLaunchKernelGGL(k_bs_gather_ties, dim3(grid_for(n)), dim3(256), 0, st, (const BRec*)R, n, (const uint64_t*)fin,
                       (const uint64_t*)lt, (const uint32_t*)(rbs + ((level - 1) & 3)), rbs + (level & 3), longrun + 1, s.err,
                       r.offs, r.bytes, level, S, pos);
    hipLaunchKernelGGL(k_bs_segsort, dim3((uint32_t)std::min<uint64_t>(4096, (m + SEG_CH - 1) / SEG_CH)), dim3(256), 0, st, S,
                       (const uint64_t*)lt, longrun, lrun, longrun + 1, lrun_cap);
    hipLaunchKernelGGL(k_bs_longsort, dim3(1024), dim3(256), 0, st, S, (const uint2*)lrun, (const unsigned int*)(longrun + 1),
                       lrun_cap);
    BRec* sorted = S;
    if (checked) {
      HIPCHK(hipMemcpyAsync(h_tot + 3, longrun, 4, hipMemcpyDeviceToHost, st));
      HIPCHK(hipStreamSynchronize(st));
      if ((uint32_t)h_tot[3]) {  // a run past RUN_LMAX: the radix passes over the whole subset
        HIPCHK(hipMemsetAsync(longrun, 0, 4, st));
        s.a = S;
        s.b = S2;
        const uint64_t top = (uint64_t)run_base + runs;  // run ids < top: bytes of run id to sort on
        const int nrb = top < (1ull << 8) ? 1 : top < (1ull << 16) ? 2 : top < (1ull << 24) ? 3 : 4;
        if ((rc = radix_sort(e, s, m, 8 + nrb, false))) return rc;
        sorted = s.a;
      }
      run_base += (uint32_t)runs;
    }
    hipLaunchKernelGGL(k_bs_put_ties, dim3(grid_for(m)), dim3(256), 0, st, (const BRec*)sorted, (const uint64_t*)lt,
                       (const uint32_t*)pos, R);
    HIPCHK(hipGetLastError());
  }
  if (!out_done) {
    if ((rc = output())) return rc;
    // complete: the callers time the sort on the host clock (ms_sort), so the
    // output kernels above must be inside it
    HIPCHK(hipMemcpyAsync(h_tot + 2, s.err, 4, hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
  }  // (else the last level's read-back came after them and read the flags)
  if ((uint32_t)h_tot[2] & 1u) return fail(MOX_EHIP, "bytewise sort: a look-back wait timed out");
  if ((uint32_t)h_tot[2] & 4u) return fail(MOX_ENOMEM, "bytewise sort: a word of 16 MiB or more (sorted on the host)");
  r.counts = oc;
  r.offs = oo;
  r.bytes = (const uint8_t*)e->s_bytes.p;
  r.sorted = true;
  return MOX_OK;
}

int bsort_table(mox_engine* e) {
  const int rc = bsort_once(e, getenv("MOX_BSORT_CHECKED") != nullptr);
  return rc == -1 ? bsort_once(e, true) : rc;
}

}  // namespace mox_host
