// Internal layout shared by the HIP kernels (mox_kernels.hip) and the host
// engine (mox_engine.hip).  Not part of the C ABI (include/mox.h).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

namespace mox {

// ---- geometry ----
constexpr int MAP_THREADS = 1024;           // 16 waves; one persistent workgroup per CU
constexpr int MAP_WG_PER_CU = 1;
constexpr int MAP_MIN_WAVES = 1;
// Ablation switches (MOX_DBG env, below) and the tools' variant builds are
// experiments: several produce wrong counts by design.  They compile only
// together with MOX_EXPERIMENT_BUILD, which tools/build_variant.sh sets and no
// product target (Makefile) does.
#if defined(MOX_ABLATE) && !defined(MOX_EXPERIMENT_BUILD)
#error "MOX_ABLATE is an experiment build (tools/build_variant.sh): not for the product library"
#endif
constexpr int MAP_LOADERS = 1;              // loader waves
#ifndef MOX_LD_SLEEP
#define MOX_LD_SLEEP 1  // k_map loader's poll for a free ring slot (s_sleep units of 64 clocks)
#endif
#ifndef MOX_CO_SLEEP
#define MOX_CO_SLEEP 1  // k_map consumer's poll for a loaded row
#endif
#ifndef MOX_RING
#define MOX_RING 32
#endif
constexpr int RING = MOX_RING;              // k_map row ring slots (LDS)
// LDS hot dictionary: single-word slots, two choices per word (dict_s1 / dict_s2,
// mox_kernels.hip); k_dict_pick picks up to DICT_MAX_WORDS candidates.
// (12-byte keys with the count inside the 16-byte slot held 4,620 words
// instead of 3,660 and cut the C2 cold records 5 %, but k_map got 15-24 us
// slower than k_reduce gained: profiles/r06/dict12_ab.txt, not kept.)
#ifndef MOX_DICT_SLOTS
#define MOX_DICT_SLOTS 5120
#endif
constexpr int DICT_SLOTS = MOX_DICT_SLOTS;
constexpr int DICT_MAX_WORDS = DICT_SLOTS < 4096 ? DICT_SLOTS : 4096;
constexpr size_t DICT_CNT_BYTES = (size_t)DICT_SLOTS * 4;  // k_map's count array
static_assert(DICT_SLOTS % 32 == 0 && DICT_SLOTS <= 65536 && DICT_MAX_WORDS <= DICT_SLOTS, "dictionary geometry");
constexpr int MAX_MAP_GRID = 1024;          // map workgroups
constexpr int MAP_WAVES = MAP_THREADS / 64;
constexpr int ROW = 1024;                   // bytes one wave classifies per step (64 lanes x 16 B)
constexpr int ROWBUF = ROW + 32;            // lowered row + 16 B look-ahead + pad (LDS)
constexpr int TOKMAX = ROW / 2;             // token starts per row (at most every other byte)
// k_map row ring (LDS): one loader wave streams rows, the other waves consume
// them.  Slot = 64 lanes x 16 B = [16 B before | PAY payload bytes | 16 B after].
constexpr int SLOT = ROW;
constexpr int PAY = ROW - 32;               // 992 payload bytes per row
constexpr int KSEL_N = 17 * 4;              // k_map key selectors: key length 0..16 x byte offset 0..3
#ifndef MOX_LD_GROUPS
#define MOX_LD_GROUPS 4  // 3: k_map +2.5-4 % on C2 (interleaved A/B)
#endif
#ifndef MOX_LD_GROUP
#define MOX_LD_GROUP 6
#endif
constexpr int LD_GROUP = MOX_LD_GROUP;      // loader: rows per register group
constexpr int LD_GROUPS = MOX_LD_GROUPS;    // groups in flight (LD_GROUP x (LD_GROUPS-1) rows outstanding)
constexpr int MAP_CONSUMERS = MAP_WAVES - MAP_LOADERS;
// (Rows loaded by their own wave by LDS-DMA, with no loader or ring, removed the
// ring's supply floor but measured 1.5-4 % slower on the whole kernel; two rows
// per wave tied with the ring at a smaller dictionary: DESIGN.md §8, round 5.)
constexpr int MAP_ROW_WAVES = MAP_CONSUMERS;  // waves that process rows
static_assert(TOKMAX - 1 >= PAY / 2, "list[TOKMAX - 1] is the token-loop sink: no row may reach it");
// A k_map token list: up to TOKMAX entries of a row, then 64 entries of tail
// (LIST_ODD, written after every row's list) that the token pass reads past
// the row's last entry instead of bounds-checking every batch
constexpr int LIST_N = TOKMAX + 64;
constexpr int NB_LOG2 = 10;                 // cold-record partitions (hash top bits)
constexpr int NB = 1 << NB_LOG2;
// k_map addresses a workgroup's NB x cold_cap cold records with 32-bit byte
// offsets (cold_at); a bigger region would need more than 4 GiB per workgroup
// (4 MiB x cold_cap over 256 workgroups: past HBM long before), and records past a
// region's end spill, so the host clamps cold_cap here
constexpr uint64_t COLD_CAP_MAX = (1ull << 32) / (16ull * NB);
constexpr uint32_t QF_MAX = 4;              // most cold regions per (map workgroup, partition) (k_map without a dictionary)
// k_map dynamic LDS (carved in this order by k_map): dictionary counts, region
// counters, misc, key selectors, dictionary keys, then the row ring with its
// ready / free words and the token lists
constexpr size_t MAP_LDS_BYTES = (size_t)DICT_SLOTS * 16 + DICT_CNT_BYTES + NB * 4 + 16 + KSEL_N * 16 +
                                 (size_t)RING * 8 + (size_t)RING * SLOT + (size_t)MAP_ROW_WAVES * 2 * LIST_N;
static_assert(MAP_LDS_BYTES <= 160 * 1024, "k_map LDS over 160 KiB");
constexpr int GC_SLOTS = 65536;             // global dictionary candidate table (k_sample -> k_dict_*)
constexpr int MAX_SAMPLE_PIECES = 1024;
constexpr int SAMPLE_PIECE = 4096;          // one 256-thread workgroup x 16 B
constexpr int SAMPLE_SLOTS = 2048;
constexpr int DH_N = 258, DH_T = 259;       // dict_hist words after the histogram and pick counters
constexpr int RED_THREADS = 1024;
// k_reduce's LDS table: RED_BK home buckets of 4 slots plus one spare bucket
// (bucket RED_BK - 1's overflow), RED_CAP distinct keys per (sub-)pass, then the
// sort scratch (slot index, RED_SORTB bins, fill cursors) and 4 counters; 2
// workgroups per CU
constexpr int RED_BK = 608;
constexpr int RED_BUCKETS = RED_BK + 1;
constexpr int RED_SLOTS = 4 * RED_BUCKETS;
constexpr int RED_CAP = 2048;
constexpr int RED_SORTB = 2048;
constexpr size_t RED_LDS_BYTES = (size_t)RED_SLOTS * (4 + 16 + 8) + RED_CAP * 2 + (RED_SORTB + 8) * 2 + RED_SORTB * 2 + 16;
static_assert(RED_SLOTS * 4 % 16 == 0 && RED_LDS_BYTES + 256 <= 80 * 1024, "k_reduce LDS: 2 workgroups per CU");
// High-cardinality split: a partition whose sampled records are
// mostly distinct is scattered into 2^kk sub-buckets (the next kk hash bits), and
// every (partition, sub-bucket) "unit" is reduced by its own workgroup.
constexpr int SUB_BITS_MAX = 12;
constexpr int SUB_N = 1 << SUB_BITS_MAX;
constexpr int U_MAX = NB * SUB_N;           // reduce units
constexpr int SUB_PER_T = SUB_N / 1024;     // sub-buckets per thread in the 1024-thread unit kernels
#ifndef MOX_SPLIT_MIN
#define MOX_SPLIT_MIN 8192
#endif
// records up to which a partition is never split: k_reduce takes it whole, in
// at most 4 table sub-passes of RED_CAP distinct keys (the exchange's reduce
// pass at C3, ~3.3 K weighted records per partition: 2048 -> 8192 took its
// span from 556 to 517 us and the N = 2 exchange from 1.07-1.10 to
// 0.86-0.88 ms, profiles/r06/split_min_ab_g31.txt)
constexpr uint32_t SPLIT_MIN = MOX_SPLIT_MIN;
constexpr uint32_t SPLIT_TARGET = 320;      // records per sub-bucket aimed at
constexpr uint32_t SMALL_CAP = 512;         // sub-buckets up to this many records: k_reduce_small
#ifndef MOX_S1_WG
#define MOX_S1_WG 4  // k_reduce_sort1 workgroups per CU (its launch bound and persistent grid; 4 -> 128 VGPRs)
#endif
#ifndef MOX_SPLIT_PER_REGION
#define MOX_SPLIT_PER_REGION 4
#endif
constexpr uint32_t SPLIT_PER_REGION = MOX_SPLIT_PER_REGION;  // sample: the first records of every map workgroup's region
constexpr uint32_t SPLIT_SAMPLE = 256 * SPLIT_PER_REGION;      // records sampled for the distinct-fraction estimate
constexpr int LC_BITS = 4096;               // linear-counting bitmap of the sample (4 bits per sample)

constexpr uint64_t LONG_TAG = 0xFF00000000000000ull;   // w1 marker of a hashed (long) key
constexpr uint64_t LONG_LEN_MASK = 0x0000FFFFFFFFFFFFull;
constexpr uint64_t ARENA_BIT = 1ull << 63;              // long-word ref points into the arena

// Ablation switches (MOX_DBG env) are compiled in only with -DMOX_ABLATE, so the
// production kernels carry no runtime debug branches (SGPR pressure in k_map).
#ifdef MOX_ABLATE
#define MOX_ABL(d, f) (((d) & (f)) != 0)
#else
#define MOX_ABL(d, f) (false)
#endif
enum : uint32_t { DBG_NO_TOKENS = 1u, DBG_NO_EMIT = 2u, DBG_NO_DICT = 4u, DBG_NO_COLDSTORE = 8u, DBG_NO_DICTADD = 16u,
                  DBG_RED_NOSORT = 32u, DBG_RED_NOINSERT = 64u, DBG_RED_NOSLOW = 128u, DBG_COUNT = 256u, DBG_RED_PLAINADD = 512u, DBG_STAMP = 1024u,
                  DBG_RED_TWICE = 2048u,    // TWICE: k_reduce streams the cold records twice (timing only: counts double)
                  DBG_NO_ROW = 4096u,       // NO_ROW: k_map consumers release each row untouched (loader + ring only)
                  DBG_PAIR_NOSTORE = 8192u, // no dictionary: pairs formed, their global stores skipped (timing only)
                  DBG_NOPAIR = 16384u,      // no dictionary: every record stored alone, no pair slots (timing A/B)
                  DBG_PAIR_SEQ = 32768u,    // no dictionary: pairs stored at consecutive addresses (timing only: wrong regions)
                  DBG_S1_SORT2 = 65536u };  // k_reduce_sort1/2 sort every unit's keys twice (timing only, same result)
// Bounds checks of derived indices (UnitDesc ranges, scatter cursors, table
// offsets), compiled in only with -DMOX_CHECK (libmox_check.so, `make check`):
// a failed check counts into ctl->dbg_cnt[0], records the largest site id in
// dbg_cnt[1], and skips the access; the host then fails the call with MOX_EHIP.
// Production builds evaluate to true and emit nothing.
enum : uint32_t {
  CHK_SMALL_DESC = 1u, CHK_SMALL_OUT = 2u, CHK_RED_OUT = 3u, CHK_SPLIT_K = 4u, CHK_SPLIT_W = 5u, CHK_UNIT = 6u,
  CHK_MAT_ROW = 7u, CHK_MAT_BYTES = 8u, CHK_SCATTER = 9u, CHK_RED_IN = 10u, CHK_GATHER = 11u,
  CHK_RED_TABLE = 12u,  // k_reduce table: a bucket's taken slots not a prefix, or one key in two slots
  CHK_RED_NU = 13u      // k_reduce: taken slots != counted new keys
};
#ifdef MOX_CHECK
#define MOX_CHK(w, ok, site) (::mox::chk_record((w).ctl, (ok), (site)))
#else
#define MOX_CHK(w, ok, site) (true)
#endif
enum : uint32_t {
  OVF_POOL = 1u, OVF_W = 2u, OVF_U = 4u, OVF_LONG = 8u, OVF_ARENA = 16u, OVF_PROBE = 32u,
  OVF_TABLE = 64u, OVF_BYTES = 128u, OVF_REDUCE = 256u, OVF_SPLIT = 512u,
  // overflows that make the records of this attempt incomplete
  OVF_RERUN = OVF_POOL | OVF_W | OVF_U | OVF_LONG | OVF_ARENA | OVF_PROBE | OVF_SPLIT
};

// Control block: counters written by the kernels, read back once per run.
struct Ctl {
  unsigned long long w_n;         // weighted records requested
  unsigned long long u_n;         // unicode tokens requested
  unsigned long long arena_n;     // arena bytes requested
  unsigned long long long_n;      // long-token inserts
  unsigned long long long_uniq;   // distinct long words (table slots claimed)
  unsigned long long tokens;
  unsigned long long err_utf8;    // min invalid byte (buffer-relative), ~0 = none
  unsigned long long halo_err;    // min token start that ran off a non-final buffer, ~0 = none
  unsigned long long cold_recs;   // records over all buckets
  unsigned long long n_short;     // distinct short words
  unsigned long long n_total;     // table entries
  unsigned long long bytes_total; // table bytes
  unsigned int overflow;
  unsigned int dict_n;
  unsigned int dict_maxprobe;
  unsigned int max_sub;
  unsigned int dict_thresh;
  unsigned int done[3];           // last-workgroup tickets: [0] k_hist
  unsigned long long cold_need;   // max records any (workgroup, partition) region asked for
  unsigned long long spill_need;  // max spill records of any map workgroup
  unsigned long long w_total;     // weighted + spilled records
  unsigned long long dbg_cnt[8];  // MOX_DBG & DBG_COUNT instrumentation
  unsigned long long n_units;     // reduce units (>= NB; > NB when partitions were split)
  unsigned long long red_ticket;  // k_reduce work queue
  unsigned long long split_k;     // cold records of split partitions
  unsigned long long split_w;     // weighted records of split partitions
  unsigned int n_split;           // partitions split
  unsigned int qf;                // cold regions per (map workgroup, partition): k_map's QF (0 = 1; mox_kernels.hip)
  unsigned long long n_big;       // entries of big_units (k_reduce work list)
  unsigned long long short_bytes; // table bytes of the short words (long words follow)
  unsigned long long n_mid;       // entries of mid_units (k_reduce_sort2 work list)
  unsigned long long n_small;     // entries of small_units (k_reduce_small work list)
  unsigned long long paths[8];    // PATH_* hit counters (MOX_PATHS builds only; zero otherwise)
  unsigned long long layout_err;  // k_map: its dynamic LDS did not start at address 0 (mox_kernels.hip L_*)
};

// ---- forced-collision check build (libmox_hc.so, `make hc`)
// -DMOX_HASH_COLLIDE truncates every key hash to a few bits, so that distinct
// words share hashes and each exactness fallback that resolves a collision by
// comparing key bytes actually runs: the 32-bit key hash (partitions,
// dictionary, reduce tables) keeps MOX_H32_BITS bits, the order hash hash32b
// MOX_H32B_BITS bits, the long-word FNV-1a-64 MOX_FNV_BITS bits.  The kept
// value is multiplied by an odd constant (a bijection), so collisions stay
// exactly as frequent while every bit position still varies (partition bits,
// dictionary slots, sub-bucket bits).  Production builds use the full hashes.
#ifdef MOX_HASH_COLLIDE
#ifndef MOX_H32_BITS
#define MOX_H32_BITS 22
#endif
#ifndef MOX_H32B_BITS
#define MOX_H32B_BITS 2
#endif
#ifndef MOX_FNV_BITS
#define MOX_FNV_BITS 8
#endif
#ifndef MOX_PATHS
#define MOX_PATHS 1
#endif
#else
#define MOX_H32_BITS 32   // unused: collide32 / fnv_finish are the identity
#define MOX_H32B_BITS 32
#endif
__host__ __device__ __forceinline__ uint32_t collide32(uint32_t h, int bits) {
#ifdef MOX_HASH_COLLIDE
  if (bits >= 32) return h;
  return (h & ((1u << bits) - 1u)) * 0x9E3779B1u;
#else
  (void)bits;
  return h;
#endif
}
// Finish of the long-word FNV-1a-64 (host and device): identity in production.
__host__ __device__ __forceinline__ uint64_t fnv_finish(uint64_t h) {
#ifdef MOX_HASH_COLLIDE
  if (MOX_FNV_BITS >= 64) return h;
  return (h & ((1ull << (MOX_FNV_BITS & 63)) - 1ull)) * 0x9E3779B97F4A7C15ull;
#else
  return h;
#endif
}
// Exactness-fallback hit counters (Ctl::paths, reported as mox_stats.path_hits):
// compiled in with -DMOX_PATHS (the collision build), so tests can assert that
// the path they target ran.
enum : uint32_t {
  PATH_DICT_SAMEHASH = 0, // k_map: a slot holds another word with the token's 32-bit hash (key compare rejects it)
  PATH_LONG_EQHASH = 1,   // long-word table: equal FNV hash, different bytes -> probe on
  PATH_SORT_RESORT = 2,   // k_reduce_sort1/2: two keys share the 23-bit sort key -> 64-bit re-sort
  PATH_SORT_TO_RED = 3,   // k_reduce_sort1/2: two keys share (h32, hash32b) -> unit goes to k_reduce
  PATH_RED_TAG = 4,       // k_reduce: table tag equal, key different
  PATH_SMALL_TAG = 5,     // k_reduce_small: hash equal, key different
  PATH_N = 8
};
#if defined(MOX_PATHS) && MOX_PATHS
#define MOX_PATH(ctlp, i) atomicAdd(&(ctlp)->paths[(i)], 1ull)
#define MOX_PATH_ADD(ctlp, i, n) atomicAdd(&(ctlp)->paths[(i)], (unsigned long long)(n))
#else
#define MOX_PATH(ctlp, i) ((void)0)
#define MOX_PATH_ADD(ctlp, i, n) ((void)0)
#endif

#ifdef MOX_CHECK
__device__ __forceinline__ bool chk_record(Ctl* ctl, bool ok, uint32_t site) {
  if (!ok) {
    atomicAdd(&ctl->dbg_cnt[0], 1ull);
    atomicMax(&ctl->dbg_cnt[1], (unsigned long long)site);
  }
  return ok;
}
#endif

// Weighted record: a key with a count (dictionary totals, spills, Unicode-lane
// short words, received partials).
struct WRec {
  uint64_t w0, w1, count;
};
// Unicode-lane token: position + length in the corpus.
struct URec {
  uint64_t pos;
  uint64_t len;
};
// Long-word table slot (all fields accessed with atomics only).
struct LSlot {
  unsigned long long h;      // hash | 1, 0 = empty
  unsigned long long ref;    // ref + 1 (0 = not yet published)
  unsigned long long len;
  unsigned long long count;
};

// ---- multi-GPU exchange ----
constexpr int MAX_RANKS = 64;
// Owner rank of a short key's partition b: ranks own contiguous partition
// ranges, so the dense table (partition order) is already in owner order.
__host__ __device__ __forceinline__ uint32_t part_owner(uint32_t b, uint32_t P) { return (uint32_t)(((uint64_t)b * P) >> NB_LOG2); }
// First partition of rank d (d may be P: returns NB).
__host__ __device__ __forceinline__ uint32_t owner_first_part(uint32_t d, uint32_t P) { return (uint32_t)(((uint64_t)d * NB + P - 1) / P); }
// Owner rank of a long word (FNV-1a-64 hash h).
__host__ __device__ __forceinline__ uint32_t long_owner(uint64_t h, uint32_t P) { return (uint32_t)(((h >> 32) * P) >> 32); }
// Long-word record header on the wire; off = byte offset of the word inside
// this (source, destination) blob's byte area, which follows the headers.
struct XHdr {
  uint64_t h, len, count, off;
};
// Per-destination counts one rank sends (one 32-byte row per peer).
struct XCnt {
  unsigned long long n_short;     // WRec records
  unsigned long long n_long;      // XHdr records
  unsigned long long long_bytes;  // word bytes, each word padded to 8
  unsigned long long pad;
};
// Kernel argument: per-peer offsets (send side: blob bases; receive side:
// blob bases + header prefix).
struct XDir {
  uint32_t P;
  uint64_t blob[MAX_RANKS + 1];   // byte offset of peer d's long blob
  uint64_t nlong[MAX_RANKS];      // headers in peer d's blob
  uint64_t hpre[MAX_RANKS + 1];   // prefix of nlong (receive side)
};

// Sorted exchange (MOX_F_SORT_BYTES at exchange time, mox_multi.hip): words
// are owned by byte range instead of by hash, so that every rank sorts its own
// words and the gather in rank order is the bytewise-sorted table.  The owner of
// a word is the number of splitters <= its first 8 bytes read big-endian (zero
// padded): bytewise order never decreases that prefix, so owners never decrease
// along the sorted table.  The splitters are quantiles of sampled prefixes of
// every rank's local table (the same on every rank).
// The splitters are weighted quantiles of sampled prefixes of every rank's
// local table (the same on every rank), chosen on the device (k_xsplit).  A
// rank's sample block: XS_SAMPLES prefixes sorted ascending, then its table
// size (the samples' weight) at XS_SAMPLES; XS_BLOCK words per block.
constexpr uint32_t XS_SAMPLES = 1024;               // sampled prefixes per rank
constexpr uint32_t XS_BLOCK = XS_SAMPLES + 8;       // block words: samples, table size, pad
constexpr uint64_t XS_NONE = ~0ull;                 // sample of an empty table (no UTF-8 word starts with 0xFF)
constexpr uint32_t XS_LDS = 16384;                  // samples k_xsplit holds (more ranks: every k-th sample)
// Skew: one prefix value holding more than XS_SKEW_NUM / XS_SKEW_DEN of a fair
// share (1 / P of the words) would load its rank past that: the exchange then
// falls back to hash owners and the gathered table is sorted at the root.
constexpr uint32_t XS_SKEW_NUM = 3, XS_SKEW_DEN = 2;
struct XSplit {
  uint32_t P;
  const uint64_t* sp;           // device: sp[0 .. P-2] ascending splitters (k_xsplit)
  uint64_t soff[MAX_RANKS];     // first record of destination d in the short send buffer
};
// owner = number of splitters <= pre, in [0, P - 1] (sp: P - 1 ascending values)
__host__ __device__ __forceinline__ uint32_t range_owner(const uint64_t* sp, uint32_t P, uint64_t pre) {
  uint32_t lo = 0, hi = P - 1;
  while (lo < hi) {
    const uint32_t mid = (lo + hi) >> 1;
    if (sp[mid] <= pre) lo = mid + 1; else hi = mid;
  }
  return lo;
}

// mox_gather: where source rank s's offsets sit in the root's receive buffer,
// and the row / byte base of its part of the gathered table.
struct GDir {
  uint32_t P;
  uint64_t roff[MAX_RANKS];
  uint64_t base_n[MAX_RANKS + 1];
  uint64_t base_b[MAX_RANKS];
  uint64_t base_b_total;
};

struct Tables {  // Unicode case data in device memory
  const uint32_t* lower_src;
  const uint32_t* lower_dst;
  const uint32_t* cased_lo;
  const uint32_t* cased_hi;
  const uint32_t* ci_lo;
  const uint32_t* ci_hi;
  int n_lower, n_cased, n_ci;
};

// Reduce unit: a whole partition (in_n == UNIT_WHOLE: its cold regions and
// weighted records) or one sub-bucket of a split partition (contiguous ranges of
// split_k / split_w).  Output: uk / uc from rec_off.
constexpr uint32_t UNIT_WHOLE = 0xFFFFFFFFu;
// u_uniq[u] flag: unit u's distinct keys are in ui[] (record index into the
// unit's split_k range + count) instead of uk[] / uc[]
constexpr uint64_t U_IDX = 1ull << 62;
struct UnitDesc {
  uint64_t in_off, win_off, rec_off;
  uint32_t in_n, win_n, part, kk;
};

struct Corpus {
  const uint8_t* base;   // 16-byte aligned
  uint64_t lo, hi;       // valid bytes [lo, hi) (internal coordinates)
  uint64_t own_lo, own_hi;
  uint64_t ctx_lo;       // own_lo == lo of corpus start? bytes < ctx_lo read as whitespace
  int at_end;
};

struct Work {  // device buffers of one engine
  Ctl* ctl;
  // dictionary
  WRec* cand;                     // GC_SLOTS candidates (key claimed with claim16, count)
  uint32_t* dict_hist;            // [256] candidate count histogram, [256] picked words (classes >= T), [257] class T - 1 words,
                                  // [DH_N] dictionary words, [DH_T] threshold (the pass's, read by k_map / k_unicode)
  WRec* dict_list;                // DICT_MAX_WORDS picked words
  uint32_t* dict_tag;             // DICT_SLOTS key hashes (0 = empty slot)
  uint4* dict_key;                // DICT_SLOTS lowered 16-byte keys
  unsigned long long* dict_tot;   // DICT_SLOTS counts summed over map workgroups
  // cold records: region (map workgroup g, partition b) = cold[(g*NB + b)*cold_cap ...]
  uint4* cold;                    // map_grid * NB * cold_cap records of 16 B
  uint32_t* cold_n;               // map_grid * NB * QF records written per region (ctl->qf regions per map workgroup)
  uint32_t* samp;                 // NB * map_grid * QF * SPLIT_PER_REGION: key hashes of every region's first records
                                  // (k_map writes them, 0 = none; k_split_count's sample)
  uint32_t cold_cap;
  uint32_t map_grid;
  uint4* spill;                   // map_grid * spill_cap records (regions that overflowed)
  uint32_t* spill_n;              // map_grid
  uint32_t spill_cap;
  // weighted records
  WRec* w;                        // w_cap
  WRec* w_sorted;                 // w_cap
  uint64_t w_cap;
  // unicode lane
  URec* u;                        // u_cap
  uint64_t u_cap;
  uint8_t* arena;                 // arena_cap
  uint64_t arena_cap;
  // long lane
  LSlot* ltab;                    // long_cap (power of two)
  uint64_t long_cap;
  // partition directory
  uint64_t* b_recs;               // NB cold records per partition
  uint32_t* b_w;                  // NB weighted records per partition
  uint32_t* b_cur;                // NB scatter cursors
  uint64_t* w_off;                // NB + 1
  uint64_t* rec_off;              // NB + 1 (output region offsets)
  uint64_t* b_uniq;               // NB
  uint64_t* uniq_off;             // NB + 1
  // reduce units (partition b = units u_base[b] .. u_base[b+1]-1; one unit
  // unless b was split into 2^b_kk[b] sub-buckets)
  uint32_t* b_kk;                 // NB
  uint32_t* red_order;            // NB: partitions by descending record count (k_unit_scan), k_reduce workgroup i takes red_order[i]
  uint32_t* u_base;               // NB + 1
  uint32_t* sub_hist;             // NB x 2 x SUB_N: cold, weighted records per sub-bucket
  uint64_t* sp_off;               // NB + 1: first split_k record of partition b
  uint64_t* spw_off;              // NB + 1: first split_w record of partition b
  UnitDesc* udesc;                // U_MAX: input ranges + output region of unit u
  uint32_t* big_units;            // U_MAX: units for k_reduce (whole partitions + oversized sub-buckets)
  uint32_t* mid_units;            // U_MAX: count-1 units of SMALL_CAP + 1 .. 2 SMALL_CAP records (k_reduce_sort2)
  uint32_t* small_units;          // U_MAX: units with weighted records, <= SMALL_CAP records (k_reduce_small)
  uint64_t* u_uniq;               // U_MAX: distinct keys of unit u
  uint64_t* u_bytes;              // U_MAX: key bytes of unit u's distinct keys
  uint64_t* u_bytes_off;          // U_MAX: byte offset of unit u inside its partition
  // table directory (k_unit_uniq_scan -> k_final_scan -> k_mat)
  uint64_t* b_bytes;              // NB: key bytes of partition b
  uint64_t* bytes_off;            // NB + 1: byte offset of partition b's first key
  uint64_t* ls_n;                 // NB: occupied long-table slots of slice b
  uint64_t* ls_b;                 // NB: bytes of slice b's long words
  uint64_t* ls_off;               // NB + 1: table index (after the short words) of slice b's first long word
  uint64_t* ls_boff;              // NB + 1: byte offset (after the short words' bytes) of slice b
  uint64_t* u_uniq_off;           // U_MAX: table index of unit u's first key inside its partition
  uint4* split_k;                 // split_k_cap cold keys grouped by unit
  WRec* split_w;                  // split_w_cap weighted records grouped by unit
  uint64_t split_k_cap, split_w_cap;
  // reduce output (capacity = records)
  uint4* uk;                      // keys
  uint64_t* uc;                   // counts
  uint32_t* ui;                   // count-1 units (k_reduce_sort1/2, u_uniq[u] & U_IDX): (record index << 16) | count
  uint64_t uniq_cap;
  // long uniques compaction
  uint64_t* lpos;                 // long_cap (scan of occupancy)
  // final table
  uint64_t* t_counts;             // table_cap
  uint64_t* t_offs;               // table_cap + 1
  uint8_t* t_bytes;               // bytes_cap
  uint64_t table_cap, bytes_cap;
  // scan scratch
  uint32_t dbg;                   // ablation switches (MOX_DBG env), 0 in production
  unsigned long long* stamps;     // DBG_STAMP: per-workgroup phase timestamps (8 per workgroup)
};

}  // namespace mox
