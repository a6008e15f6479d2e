// HIP kernels of the MI355X word-count engine (gfx950 / CDNA4, wave64).
//
// Hot path of the reference (/root/reference/src/main.rs:16-22):
//   split_file (:36-51) -> map_phase/count_words (:53-101) -> write/read map files
//   (:103-109, :152-168) -> reduce_phase (:111-150)
// re-designed as (DESIGN.md has the data layout and rooflines):
//   k_sample + k_dict_*       hot-word dictionary from a 192 x 4 KiB sample
//   k_map                     one streaming pass over the corpus in HBM: 16 B/lane
//                             coalesced loads, ASCII fast path (SWAR whitespace /
//                             case classification, per-lane token extraction from a
//                             32-byte window), UTF-8 validation + Unicode whitespace
//                             on tiles with non-ASCII bytes, hot words counted in an
//                             LDS dictionary, all other words emitted as exact 16-byte
//                             keys into 1024 hash partitions
//                             (= the shuffle write, main.rs:103-109)
//   k_unicode                 full Unicode lowercase + Final_Sigma for non-ASCII tokens,
//                             and the dictionary totals as weighted records
//   k_hist (+ bucket scan in its last workgroup), k_scatter   shuffle directory
//   k_split_count, k_unit_scan, k_split_scatter
//                             high-cardinality split of partitions into sub-bucket units
//   k_reduce, k_reduce_small  per-unit LDS hash group-by / sort-based reduce (= reduce_phase merge,
//                             main.rs:132-134), deterministic (hash, key) order
//   long table                words > 16 bytes: hashed keys, byte-compare resolution
//   k_unit_uniq_scan, k_final_scan, k_mat
//                             dense (word, count) table in HBM, one pass
#include "mox_internal.h"

namespace mox {

// ------------------------------------------------------------------ helpers
// per-byte masks, valid only when every byte < 0x80 (ASCII fast path)
__device__ __forceinline__ uint32_t movemask8(uint64_t m80) {  // m80: 0x80 per selected byte
  uint64_t m = (m80 >> 7) & 0x0101010101010101ull;  // bit 8i = byte i
  m |= m >> 7;   // bits 0,1 | 16,17 | 32,33 | 48,49
  m |= m >> 14;  // bits 0..3 | 32..35
  m |= m >> 28;  // bits 0..7
  return (uint32_t)m & 0xFFu;
}
__device__ __forceinline__ uint64_t zero_bytes80(uint64_t v) {  // exact: 0x80 where byte == 0
  uint64_t t = (v & 0x7F7F7F7F7F7F7F7Full) + 0x7F7F7F7F7F7F7F7Full;
  return ~(t | v | 0x7F7F7F7F7F7F7F7Full);
}
__device__ __forceinline__ uint64_t ws_bytes80(uint64_t x) {  // ASCII whitespace 09..0D, 20
  uint64_t sp = zero_bytes80(x ^ 0x2020202020202020ull);
  uint64_t ge9 = x + 0x7777777777777777ull;   // b + 0x77 >= 0x80  <=> b >= 9
  uint64_t ge14 = x + 0x7272727272727272ull;  // b >= 14
  return (sp | (ge9 & ~ge14)) & 0x8080808080808080ull;
}
__device__ __forceinline__ uint64_t lower_ascii(uint64_t x) {
  uint64_t ge_a = x + 0x3F3F3F3F3F3F3F3Full;  // b >= 'A'
  uint64_t gt_z = x + 0x2525252525252525ull;  // b >= 'Z'+1
  return x | (((ge_a & ~gt_z) & 0x8080808080808080ull) >> 2);
}
__device__ __forceinline__ bool is_ascii_ws(uint32_t b) { return b == 0x20 || (b >= 9 && b <= 13); }
__device__ __forceinline__ uint8_t ascii_lower(uint8_t b) { return (b >= 'A' && b <= 'Z') ? (uint8_t)(b + 32) : b; }
__device__ __forceinline__ uint64_t fnv_step(uint64_t h, uint8_t b) { return (h ^ b) * 0x100000001b3ull; }
constexpr uint64_t FNV0 = 0xcbf29ce484222325ull;

__device__ __forceinline__ uint64_t lo_mask(int nbytes) {  // 0 <= nbytes <= 8
  return nbytes >= 8 ? ~0ull : ((1ull << (8 * nbytes)) - 1);
}

// Exclusive scan of one value per thread over a 1024-thread workgroup.
__device__ __forceinline__ uint64_t block_exscan(uint64_t x, uint64_t* wsum, uint64_t& total) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nw = blockDim.x >> 6;
  uint64_t incl = x;
  for (int off = 1; off < 64; off <<= 1) {
    const uint64_t y = __shfl_up(incl, off);
    if (lane >= off) incl += y;
  }
  if (lane == 63) wsum[wv] = incl;
  __syncthreads();
  uint64_t pre = 0, tot = 0;
  for (int k = 0; k < nw; k++) { const uint64_t t = wsum[k]; if (k < wv) pre += t; tot += t; }
  __syncthreads();
  total = tot;
  return pre + incl - x;
}

// Last-workgroup handoff: true in the one workgroup of the grid that takes the
// last ticket.  The words that workgroup reads from the others are published
// with agent-scope atomics (RMW or st_agent), which are performed past the
// XCD-private L2s: no cache write-back, only a wait for them to complete before
// the ticket (a __threadfence() here would write back L2 in every workgroup).
// The last workgroup reads them with ld_agent.  `ticket` is a Ctl word zeroed
// by k_init; every workgroup of the grid must call this (no early return).
template <class T>
__device__ __forceinline__ void st_agent(T* p, T v) { __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
template <class T>
__device__ __forceinline__ T ld_agent(const T* p) { return __hip_atomic_load(const_cast<T*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT); }
__device__ __forceinline__ bool last_block(unsigned int* ticket) {
  __shared__ bool s_last;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // this thread's atomics are performed
  __syncthreads();
  if (threadIdx.x == 0) s_last = __hip_atomic_fetch_add(ticket, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == gridDim.x - 1;
  __syncthreads();
  return s_last;
}

// Corpus byte with out-of-range bytes reading as ' ' (whitespace).
__device__ __forceinline__ uint8_t byte_at(const Corpus& c, uint64_t p) {
  if (p < c.lo || p >= c.hi) return 0x20;
  return c.base[p];
}

// Length of the Unicode White_Space char starting at p (0 if none), valid UTF-8 assumed.
// Rust char::is_whitespace: 09-0D 20 | 85 A0 | 1680 | 2000-200A 2028 2029 202F 205F | 3000
__device__ __forceinline__ int ws_len_at(const Corpus& c, uint64_t p) {
  uint8_t b0 = byte_at(c, p);
  if (b0 < 0x80) return is_ascii_ws(b0) ? 1 : 0;
  if (b0 != 0xC2 && b0 != 0xE1 && b0 != 0xE2 && b0 != 0xE3) return 0;
  uint8_t b1 = byte_at(c, p + 1);
  if (b0 == 0xC2) return (b1 == 0x85 || b1 == 0xA0) ? 2 : 0;
  uint8_t b2 = byte_at(c, p + 2);
  if (b0 == 0xE1) return (b1 == 0x9A && b2 == 0x80) ? 3 : 0;
  if (b0 == 0xE3) return (b1 == 0x80 && b2 == 0x80) ? 3 : 0;
  if (b1 == 0x80) return ((b2 >= 0x80 && b2 <= 0x8A) || b2 == 0xA8 || b2 == 0xA9 || b2 == 0xAF) ? 3 : 0;
  if (b1 == 0x81) return b2 == 0x9F ? 3 : 0;
  return 0;
}
// Is byte p part of a whitespace char?
__device__ __forceinline__ bool in_ws(const Corpus& c, uint64_t p) {
  if (p < c.lo || p >= c.hi) return true;
  if (ws_len_at(c, p) >= 1) return true;
  if (p >= 1 && ws_len_at(c, p - 1) >= 2) return true;
  if (p >= 2 && ws_len_at(c, p - 2) >= 3) return true;
  return false;
}
__device__ __forceinline__ int lead_len(uint8_t b) {
  if (b < 0x80) return 1;
  if (b >= 0xC2 && b <= 0xDF) return 2;
  if (b >= 0xE0 && b <= 0xEF) return 3;
  if (b >= 0xF0 && b <= 0xF4) return 4;
  return 0;  // continuation or never-valid byte
}
// UTF-8 validity of the byte at p (Rust core::str::from_utf8 rules), given
// neighbours up to 3 bytes away.  Returns 0 ok, 1 invalid, 2 needs more halo.
__device__ int utf8_check(const Corpus& c, uint64_t p) {
  uint8_t b = c.base[p];
  bool cont = (b & 0xC0) == 0x80;
  bool must = false;
  for (int k = 1; k <= 3; k++) {
    if (p < c.lo + (uint64_t)k) break;
    uint8_t q = c.base[p - k];
    if (lead_len(q) > k && q >= 0xC0) { must = true; break; }
  }
  if (cont != must) return 1;
  if (cont || b < 0x80) return 0;
  int L = lead_len(b);
  if (L == 0) return 1;
  if (p + (uint64_t)L > c.hi) return c.at_end ? 1 : 2;
  uint8_t b1 = c.base[p + 1];
  if (b == 0xE0 && b1 < 0xA0) return 1;
  if (b == 0xED && b1 > 0x9F) return 1;
  if (b == 0xF0 && b1 < 0x90) return 1;
  if (b == 0xF4 && b1 > 0x8F) return 1;
  return 0;
}

// ------------------------------------------------------------------ long lane
// Lowered byte i of a long word reference (corpus refs are ASCII tokens).
__device__ __forceinline__ uint8_t ref_byte(const uint8_t* base, const uint8_t* arena, uint64_t ref, uint64_t i) {
  if (ref & ARENA_BIT) return arena[(ref & ~ARENA_BIT) + i];
  return ascii_lower(base[ref + i]);
}
__device__ bool long_equal(const uint8_t* base, const uint8_t* arena, uint64_t ra, uint64_t rb, uint64_t len) {
  for (uint64_t i = 0; i < len; i++)
    if (ref_byte(base, arena, ra, i) != ref_byte(base, arena, rb, i)) return false;
  return true;
}
// Exact insert into the long-word table; every access is an atomic (memory-side,
// coherent across XCDs).  Keys: (hash, len) + byte compare on hash equality.
// A wave-level loop (as cold_pair's): every lane takes one probe step per
// iteration and the body ends in a wave barrier, so a lane that claims a slot
// publishes it inside that iteration.  In a lane-level loop the compiler may
// sink the claimant's publication (code reached only on the exit path) past the
// loop exit, where it waits for lanes of its own wave that spin on that very
// publication: the forced-collision build (-DMOX_HASH_COLLIDE) lost the counts
// of repeated long words that way.
template <class W>  // Work, or the kernarg-segment Work of k_map's rare paths
__device__ void long_insert(const W& w, const uint8_t* base, uint64_t h, uint64_t ref, uint64_t len, uint64_t cnt) {
  h |= 1;
  const uint64_t mask = w.long_cap - 1;
  uint64_t slot = h & mask, probes = 0;
  uint32_t spins = 0, eqh = 0;
  bool done = false;
  do {
    if (!done) {
      if (++spins > (1u << 24)) {
        atomicOr(&w.ctl->overflow, OVF_PROBE);
        done = true;
      } else {
        LSlot* s = &w.ltab[slot];
        const unsigned long long cur = atomicCAS(&s->h, 0ull, (unsigned long long)h);
        bool next = false;
        if (cur == 0) {
          // publish len before ref: memory-side atomics to different words complete
          // in any order, so the fence (s_waitcnt vmcnt(0)) orders them
          atomicExch(&s->len, (unsigned long long)len);
          __threadfence();
          atomicExch(&s->ref, (unsigned long long)(ref + 1));
          atomicAdd(&s->count, (unsigned long long)cnt);
          atomicAdd(&w.ctl->long_uniq, 1ull);
          done = true;
        } else if (cur == h) {
          const unsigned long long r = atomicAdd(&s->ref, 0ull);
          if (r != 0) {  // (0: the claimant is still publishing -- this slot again next iteration)
            // acquire: the claimant's arena bytes (written before its release fence,
            // possibly from another XCD's L2) must be seen before they are compared
            __atomic_thread_fence(__ATOMIC_ACQUIRE);
            const unsigned long long l = atomicAdd(&s->len, 0ull);
            if (l == len && long_equal(base, w.arena, r - 1, ref, len)) {
              atomicAdd(&s->count, (unsigned long long)cnt);
              done = true;
            } else {
              eqh++;  // same hash, another word: probe on
              next = true;
            }
          }
        } else {
          next = true;
        }
        if (next) {
          slot = (slot + 1) & mask;
          if (++probes > mask) {
            atomicOr(&w.ctl->overflow, OVF_LONG);
            done = true;
          }
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  } while (__any(!done));
  // the path counter is added once, after the loop: an atomic on it inside the
  // loop next to the slot-count add (both "+1" in k_unicode) was merged by the
  // compiler (ROCm 7.2) into one atomic whose address lost the slot-count case
  // -- repeated long words' counts went to the counter
  if (eqh) MOX_PATH_ADD(w.ctl, PATH_LONG_EQHASH, eqh);
  (void)eqh;
}

// ------------------------------------------------------------------ map kernel
// 32-bit key hash of a short (<= 16 byte) key given as 4 little-endian dwords:
// a multiply/xor fold then a two-round multiply-xorshift finaliser.  Bit use:
// partition = top NB_LOG2 bits, dictionary home slot = low 12 bits, second
// dictionary group = bits 12..21; reduce slots use a multiplicative hash of all
// bits.  Final table order is (h32, hash32b, key) (key_less), so it is deterministic.
// The fold: k0 ^ k1 C ^ rotl(k2, 21) ^ rotl(k3, 6) (C odd: the product a
// bijection of k1), one v_mul_lo_u32, two v_alignbit and one 3-input v_bitop3
// + xor.  Until round 5 k1 was rotated by 11 instead of multiplied, the same
// instruction count, but the fold was then linear over GF(2) on ASCII bytes
// whose high bits agree: over the ZIPF vocabulary's 3.76 M keys (with trailing
// marks) it gave 173,889 colliding pairs against ~1,650 for a random 32-bit
// hash (this fold: 2,353; three multiplies: 1,768, but k_map +1.5 %); HICARD-
// like keys 8,031 against ~1,180 (this: 1,198).  Equal hashes of different
// keys are correct everywhere but slow: k_reduce sent ~275 K records per C2
// pass to its insert loop on them (profiles/r05/hash_fold_collisions.txt).
__device__ __forceinline__ uint32_t hash_fold(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  return __builtin_amdgcn_bitop3_b32(k0, k1 * 0x85EBCA77u, __builtin_rotateleft32(k2, 21), 0x96) ^ __builtin_rotateleft32(k3, 6);
}
// The finaliser, a bijection of the fold (collisions are the fold's alone).
// MOX_HASH_FIN1: one multiply-xorshift round, a * C ^ (a * C) >> 16: its top
// bits (partition), low and high 16 bits (dictionary slots, k_reduce bucket)
// are as uniform over the ZIPF vocabulary as the two-round finaliser's
// (chi2 / dof 0.89-1.03, tools/hash_collisions.py's keys), three VALU fewer.
#ifndef MOX_HASH_FIN1
#define MOX_HASH_FIN1 1
#endif
__device__ __forceinline__ uint32_t hash_fin(uint32_t a) {
  a *= 0x9E3779B1u;
  if (MOX_HASH_FIN1) return a ^ (a >> 16);
  a ^= a >> 15;
  a *= 0x85EBCA6Bu;
  return a ^ (a >> 13);
}
__device__ __forceinline__ uint32_t hash32(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  const uint32_t a = hash_fin(hash_fold(k0, k1, k2, k3));
  // never 0: 0 marks a free slot in the dictionary and k_reduce tag arrays (a
  // key hashing to 0 would spin on a "free" slot); 1 simply shares its hash
  return max(collide32(a, MOX_H32_BITS), 1u);  // collide32: identity except in the collision build
}
// k_map's token passes: hash32 without the max (one VALU instruction per key
// less).  It differs from hash32 only where hash32 is 1 and this is 0, which
// give the same partition (top bits) and dictionary slots (dict_s1 / dict_s2 of
// 0 and 1 are both 0), so cold records and dictionary probes agree with every
// other kernel; where k_map stores the hash itself (note_sample: 0 = no
// record) it takes the max.  (Setting bit 0 instead, (a ^ a >> 13) | 1 in one
// v_bitop3, changed the low bits k_reduce's slot choice uses: k_reduce +4 %.)
__device__ __forceinline__ uint32_t hash32_map(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
#ifdef MOX_HASH_COLLIDE
  return hash32(k0, k1, k2, k3);
#else
  return hash_fin(hash_fold(k0, k1, k2, k3));
#endif
}
__device__ __forceinline__ uint32_t key_hash(uint64_t w0, uint64_t w1) {
  return hash32((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
}
__device__ __forceinline__ uint32_t bucket_of(uint32_t h) { return h >> (32 - NB_LOG2); }
// Cold-record regions.  Map workgroup g writes partition b's records to its
// region (g, b).  Without a dictionary (high-cardinality input) it keeps QF
// regions per partition instead, one per value q of the log2(QF) hash bits
// right below the partition bits, of cold_cap / QF records each, so that
// k_split_scatter can move a partition one q-slice at a time (a QF-th of its
// sub-buckets open at once).  Readers see RG = QF x map_grid regions per
// partition ("virtual map workgroups" g' = QF g + q) of RC = cold_cap / QF
// records: region (g', b) starts at cold + (g' NB + b) RC.  k_map records QF
// in ctl->qf (0 = 1: dictionary passes and reduce-only passes).
__device__ __forceinline__ uint32_t hc_qf(uint32_t map_grid) {
  return map_grid * 4u <= (uint32_t)MAX_MAP_GRID ? 4u : (map_grid * 2u <= (uint32_t)MAX_MAP_GRID ? 2u : 1u);
}
__device__ __forceinline__ uint32_t reg_qf(const Work& w) { const uint32_t q = w.ctl->qf; return q ? q : 1u; }
__device__ __forceinline__ uint32_t reg_grid(const Work& w) { return w.map_grid * reg_qf(w); }
__device__ __forceinline__ uint32_t reg_cap(const Work& w) { return w.cold_cap / reg_qf(w); }
// Records written into region (g, b) of a grid of RG regions per partition.
// Partition-major (b RG + g): a partition's row is contiguous for k_hist's
// sums, k_reduce's region prefix and the split kernels' region lists.
__device__ __forceinline__ uint32_t& cold_n_at(const Work& w, uint32_t RG, uint32_t g, uint32_t b) {
  return w.cold_n[(uint64_t)b * RG + g];
}
// byte length of a short key (lowered word, zero padded to 16 bytes, no NUL inside)
__device__ __forceinline__ uint32_t key_len16(uint4 k) {
  const uint64_t w0 = ((uint64_t)k.y << 32) | k.x, w1 = ((uint64_t)k.w << 32) | k.z;
  if (w1) return 16 - (__clzll(w1) >> 3);
  return 8 - (__clzll(w0) >> 3);
}
// Dictionary: DICT_SLOTS single-word slots, two choices per word (s1 from the
// low 16 hash bits, s2 from the high 16).  k_dict_build places the words hottest
// first into s1, else s2, else leaves the word cold (2-choice greedy: ~98 % of
// the picked words' sampled tokens placed).  The token pass reads both slots'
// keys at once and compares them with the token's key, so a lookup is one LDS
// round trip and decides the token: a hit counts in LDS, a miss is cold.  No
// tags, no second probe pass.
__device__ __forceinline__ uint32_t dict_s1(uint32_t h) { return ((h & 0xFFFFu) * (uint32_t)DICT_SLOTS) >> 16; }
__device__ __forceinline__ uint32_t dict_s2(uint32_t h) { return ((h >> 16) * (uint32_t)DICT_SLOTS) >> 16; }
// k_map's token pass: a slot's key byte offset (16 B keys), dict_s1 / dict_s2
// scaled, from the fastrange product p in one v_lshlrev_b32_sdwa ((p >> 16) << 4:
// the shift reads p's high half).  Left to the compiler it took two
// instructions, since the slot also addressed the count array.
__device__ __forceinline__ uint32_t slot_off16(uint32_t p) {
  uint32_t r;
  asm("v_lshlrev_b32_sdwa %0, 4, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:WORD_1" : "=v"(r) : "v"(p));
  return r;
}

// LDS pair slot states (k_map without a dictionary, k_split_scatter): a
// record waits in its slot until the next record for the same region arrives,
// and the pair goes out as one aligned 32-byte sector.
constexpr uint32_t PS_EMPTY = 0u, PS_BUSY = 1u, PS_FULL = 2u;
struct MapLds {
  uint4* dkey;      // DICT_SLOTS 16-byte keys (zero = empty: a real key is never zero)
  uint32_t* dcnt;   // DICT_SLOTS
  uint32_t* bcnt;   // NB x qf: cold records this workgroup wrote per region (no dictionary: inside dcnt's space)
  uint32_t* misc;   // [0] spills [1] row ticket
  uint4* seltab;    // [KSEL_N]: v_perm selectors of a len-byte key at byte offset sh (entry 4 len + sh)
  uint32_t kmask;   // 0x3FC in a VGPR (key_load's v_bitop3_b32 takes no literal)
  // no dictionary (dict_n == 0): pair slots per region, inside dkey's space
  uint4* pend;      // NB x qf parked records
  uint32_t* pst;    // NB x qf slot states (PS_*)
};

// k_map LDS layout: byte offsets from the dynamic LDS base, which is address 0
// (k_map has no static LDS; checked at entry, Ctl::layout_err).  As constants
// the compiler folds them into the LDS instructions' 16-bit offset field (from
// the extern array's symbol it added the base per access, v_add_u32 v, 0, v).
// The row ring comes first, so every row slot is SLOT-aligned and key_load ORs
// a token's 4-aligned offset into its slot address (v_and_or_b32).
constexpr uint32_t L_ROWS = 0;
constexpr uint32_t L_ROWS_BYTES = RING * SLOT;
constexpr uint32_t L_DCNT = L_ROWS + L_ROWS_BYTES;
constexpr uint32_t L_BCNT = L_DCNT + (uint32_t)DICT_CNT_BYTES;
constexpr uint32_t L_MISC = L_BCNT + NB * 4;
constexpr uint32_t L_SELTAB = L_MISC + 16;
constexpr uint32_t L_DKEY = L_SELTAB + KSEL_N * 16;
constexpr uint32_t L_RFLAGS = L_DKEY + DICT_SLOTS * 16;  // ring: ready[RING], free[RING]
constexpr uint32_t L_LISTS = L_RFLAGS + RING * 8u;
static_assert(L_LISTS + (size_t)MAP_ROW_WAVES * 2 * LIST_N == MAP_LDS_BYTES, "k_map LDS layout");
static_assert(L_ROWS % SLOT == 0 && (SLOT & (SLOT - 1)) == 0, "row slots aligned to their size");
static_assert(L_DCNT % 16 == 0 && L_SELTAB % 16 == 0 && L_DKEY % 16 == 0 && L_LISTS % 16 == 0, "LDS table alignment");
typedef __attribute__((address_space(3))) uint8_t LdsByte;
// LDS address of a generic pointer into LDS, and a pointer from an LDS address
__device__ __forceinline__ uint32_t lds_addr(const void* p) { return (uint32_t)(uintptr_t)(const LdsByte*)p; }
template <class T>
__device__ __forceinline__ T* lds_ptr(uint32_t a) {
  return (T*)(__attribute__((address_space(3))) T*)(uintptr_t)a;
}

typedef const __attribute__((address_space(4))) Work* KWork;  // constant (kernarg) address space: scalar loads
struct MapCtx {
  Corpus c;
  Work w;            // hot path: cold, cold_cap only
  KWork wk;          // the kernel argument itself (kernarg segment), for the rare paths
  MapLds s;
  uint32_t dict_n;
  uint32_t qf, qb;   // regions per partition (QF, 1 with a dictionary) and log2(qf)
  uint32_t rg, rc;   // regions per partition over the grid (qf map_grid), records per region (cold_cap / qf)
  uint4* wcold;      // this workgroup's first region (q = 0, b = 0): cold + blockIdx qf NB rc
  uint32_t keep;     // do_row: ~0 in lanes 1..62, 0 in the context lanes 0 and 63 (opaque VGPR)
};
// Record pos of this workgroup's region q of partition b: one 64-bit
// multiply-add and one address add from the workgroup's region base (the
// full region index needed four more instructions per cold store)
// A workgroup's regions span NB cold_cap records (cold_cap <= COLD_CAP_MAX), so
// the byte offset fits 32 bits: one v_mad_u32_u24 and a shift, and the store
// takes the 64-bit base from SGPRs (a v_mad_u64_u32 and two v_lshl_add_u64 in
// 64-bit form)
__device__ __forceinline__ uint4* cold_at(const MapCtx& m, uint32_t b, uint32_t q, uint32_t pos) {
  return reinterpret_cast<uint4*>(reinterpret_cast<uint8_t*>(m.wcold) + ((__umul24(q * NB + b, m.rc) + pos) << 4));
}
// Work fields of the rare paths (spills, Unicode lane, long words, error
// flags), loaded where they are used: the opaque pointer keeps the compiler from
// hoisting these loads to the kernel entry, where ~20 more SGPRs would stay live
// across the row loop and spill into VGPR lanes (v_readlane in the hot path).
__device__ __forceinline__ KWork rare_ptr(const MapCtx& m) {
  KWork p = m.wk;
  asm volatile("" : "+s"(p));
  return p;
}
#define rare(m) (*rare_ptr(m))

__device__ __forceinline__ bool key_eq(uint4 k, uint64_t w0, uint64_t w1) {
  return k.x == (uint32_t)w0 && k.y == (uint32_t)(w0 >> 32) && k.z == (uint32_t)w1 && k.w == (uint32_t)(w1 >> 32);
}
// Exact dictionary lookup: the key's two slots.
__device__ __forceinline__ int dict_find(const MapLds& s, uint32_t h, uint64_t w0, uint64_t w1) {
  const uint32_t s1 = dict_s1(h), s2 = dict_s2(h);
  if (key_eq(s.dkey[s1], w0, w1)) return (int)s1;
  if (key_eq(s.dkey[s2], w0, w1)) return (int)s2;
  return -1;
}

__device__ __forceinline__ void cold_word(const MapCtx& m, uint32_t h, uint64_t w0, uint64_t w1);

// A short word (lowered length <= 16, no NUL byte) as an exact 16-byte key.
// Hot words: LDS dictionary count.  Others: appended to this workgroup's
// region of the word's partition (the shuffle write), no global atomics.
__device__ __forceinline__ void short_word(const MapCtx& m, uint64_t w0, uint64_t w1) {
  const uint32_t h = key_hash(w0, w1);
  if MOX_ABL(m.w.dbg, DBG_NO_EMIT) { asm volatile("" ::"v"(h)); return; }
  if (m.dict_n && !MOX_ABL(m.w.dbg, DBG_NO_DICT)) {
    const int slot = dict_find(m.s, h, w0, w1);
    if (slot >= 0) {
      if (!MOX_ABL(m.w.dbg, DBG_NO_DICTADD)) atomicAdd(&m.s.dcnt[slot], 1u);
      return;
    }
  }
  cold_word(m, h, w0, w1);
}

// A word not in the dictionary: appended to this workgroup's region of its
// hash partition (the shuffle write), no global atomics.
__device__ __forceinline__ void cold_spill(const MapCtx& m, uint4 key) {
  const uint32_t sp = atomicAdd(&m.s.misc[0], 1u);
  if (sp < rare(m).spill_cap) {
    rare(m).spill[(uint64_t)blockIdx.x * rare(m).spill_cap + sp] = key;
    return;
  }
  atomicOr(&rare(m).ctl->overflow, OVF_POOL);
}
// No dictionary: records go out in pairs (one aligned 32-byte sector each; a
// lone 16-byte store costs the memory a read-modify-write).  Three-state LDS
// slot per partition; a lane that finds it BUSY retries, and the BUSY holder
// finishes within the same loop iteration, so no lane waits on another's
// progress.  Regions start at even records (cold_cap is even).
// One attempt of the pair protocol on slot `slot` for record k: true when the
// record was parked or paired.  *q gets the parked partner when paired.
__device__ __forceinline__ int pair_try(uint32_t* pst, uint4* pend, uint32_t slot, uint4 k, uint4* q) {
  uint32_t st = PS_EMPTY;
  if (__hip_atomic_compare_exchange_strong(&pst[slot], &st, PS_BUSY, __ATOMIC_ACQUIRE, __ATOMIC_RELAXED,
                                           __HIP_MEMORY_SCOPE_WORKGROUP)) {
    pend[slot] = k;
    __hip_atomic_store(&pst[slot], PS_FULL, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return 1;  // parked
  }
  if (st == PS_FULL && __hip_atomic_compare_exchange_strong(&pst[slot], &st, PS_BUSY, __ATOMIC_ACQUIRE,
                                                            __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {
    *q = pend[slot];
    __hip_atomic_store(&pst[slot], PS_EMPTY, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_WORKGROUP);
    return 2;  // paired with *q
  }
  return 0;  // BUSY: retry
}
// The retry loop is a wave-level loop (exit when no lane is left) whose body
// ends in a wave barrier: a lane's slot stores stay inside the iteration in
// which it won the slot.  (A per-lane `while (!done)` loop lets the compiler
// sink them past the loop exit, where the winning lane waits for the spinning
// lanes of its own wave: a SIMT deadlock.)
// k_split_count's sample: the key hashes of the first SPLIT_PER_REGION records
// of every (workgroup, partition) region, written when a record lands at such a
// position (rare: 4 of ~150 records per region at C2), so that the split
// decision reads 4 KiB per partition instead of 1,024 scattered records.
__device__ __forceinline__ void note_sample(const MapCtx& m, uint32_t b, uint32_t q, uint32_t pos, uint32_t h) {
  if (pos < SPLIT_PER_REGION)
    rare(m).samp[((uint64_t)b * m.rg + blockIdx.x * m.qf + q) * SPLIT_PER_REGION + pos] = h;
}
// No dictionary: slot B = the partition bits and the qb bits below them
// (partition b = B >> qb, region q = B & (qf - 1)).
__device__ __forceinline__ void cold_pair(const MapCtx& m, uint32_t B, uint32_t h, uint4 key) {
  const uint32_t b = B >> m.qb, qr = B & (m.qf - 1);
  bool done = false;
  do {
    if (!done) {
      uint4 q;
      const int r = pair_try(m.s.pst, m.s.pend, B, key, &q);
      if (r == 2) {
        const uint32_t pos = atomicAdd(&m.s.bcnt[B], 2u);
        if (MOX_ABL(m.w.dbg, DBG_PAIR_NOSTORE)) {
          asm volatile("" ::"v"(pos), "v"(q.x));
        } else if (MOX_ABL(m.w.dbg, DBG_PAIR_SEQ)) {
          const uint64_t slab = (uint64_t)NB * m.qf * m.rc;
          const uint32_t sp = atomicAdd(&m.s.misc[2], 2u) % (uint32_t)(slab > 0xFFFFFFF0ull ? 0xFFFFFFF0ull : slab - 1);
          uint4* o = m.w.cold + blockIdx.x * slab + (sp & ~1u);
          o[0] = q;
          o[1] = key;
        } else {
          if (pos < SPLIT_PER_REGION) {
            note_sample(m, b, qr, pos, hash32(q.x, q.y, q.z, q.w));
            note_sample(m, b, qr, pos + 1, max(h, 1u));  // (h: hash32_map)
          }
          if (pos + 1 < m.rc) {
            uint4* o = cold_at(m, b, qr, pos);
            o[0] = q;
            o[1] = key;
          } else {
            cold_spill(m, q);
            cold_spill(m, key);
          }
        }
      }
      done = r != 0;
    }
    __builtin_amdgcn_wave_barrier();
  } while (__any(!done));
}
__device__ __forceinline__ void cold_word(const MapCtx& m, uint32_t h, uint64_t w0, uint64_t w1) {
  const uint32_t b = bucket_of(h);
  if MOX_ABL(m.w.dbg, DBG_NO_COLDSTORE) { asm volatile("" ::"v"(b)); return; }
  const uint4 key = make_uint4((uint32_t)w0, (uint32_t)(w0 >> 32), (uint32_t)w1, (uint32_t)(w1 >> 32));
  if (m.dict_n == 0) {
    if (!MOX_ABL(m.w.dbg, DBG_NOPAIR)) { cold_pair(m, h >> (32 - NB_LOG2 - m.qb), h, key); return; }
    const uint32_t B = h >> (32 - NB_LOG2 - m.qb), qr = B & (m.qf - 1);
    const uint32_t pos = atomicAdd(&m.s.bcnt[B], 1u);
    if (pos < SPLIT_PER_REGION) note_sample(m, b, qr, pos, max(h, 1u));  // (h: hash32_map)
    if (pos < m.rc) *cold_at(m, b, qr, pos) = key;
    else cold_spill(m, key);
    return;
  }
  const uint32_t pos = atomicAdd(&m.s.bcnt[b], 1u);
  if (pos < SPLIT_PER_REGION) note_sample(m, b, 0, pos, max(h, 1u));  // (h: hash32_map)
  if (pos < m.rc) {
    *cold_at(m, b, 0, pos) = key;
    return;
  }
  cold_spill(m, key);
}

// Any token, walked byte by byte from global memory (rare: long tokens, tokens
// running past the look-ahead window, rows with non-ASCII bytes).
__device__ void generic_token(const MapCtx& m, uint64_t p) {
  const Corpus& c = m.c;
  uint64_t q = p;
  bool nonascii = false, nul = false;
  for (;;) {
    if (q >= c.hi) {
      if (!c.at_end) atomicMin(&rare(m).ctl->halo_err, (unsigned long long)(p - c.lo));
      break;
    }
    const uint8_t b = c.base[q];
    if (b < 0x80) {
      if (is_ascii_ws(b)) break;
      nul |= (b == 0);
      q++;
    } else {
      if (ws_len_at(c, q)) break;
      nonascii = true;
      q++;
    }
  }
  const uint64_t len = q - p;
  if (nonascii) {
    const unsigned long long i = atomicAdd(&rare(m).ctl->u_n, 1ull);
    if (i < rare(m).u_cap) rare(m).u[i] = URec{p, len};
    else atomicOr(&rare(m).ctl->overflow, OVF_U);
    return;
  }
  if (len <= 16 && !nul) {
    uint64_t w0 = 0, w1 = 0;
    for (uint64_t i = 0; i < len; i++) {
      const uint64_t b = ascii_lower(c.base[p + i]);
      if (i < 8) w0 |= b << (8 * i); else w1 |= b << (8 * (i - 8));
    }
    short_word(m, w0, w1);
    return;
  }
  uint64_t h = FNV0;
  for (uint64_t i = 0; i < len; i++) h = fnv_step(h, ascii_lower(c.base[p + i]));
  h = fnv_finish(h);
  atomicAdd(&rare(m).ctl->long_n, 1ull);
  long_insert(rare(m), c.base, h, p, len, 1);
}

// Clamped aligned 16-byte load: the block always overlaps [lo, hi), so it never
// leaves the allocation; bytes out of range are fixed up by fix16.
__device__ __forceinline__ uint4 raw16(const Corpus& c, uint64_t p) {
  // an empty buffer has no block to clamp to (c.hi - 1 < c.lo: the clamp would
  // land 16 bytes below the buffer): read nothing
  if (c.hi <= c.lo) return make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
  const uint64_t first = c.lo & ~15ull, last = (c.hi - 1) & ~15ull;
  p = p < first ? first : (p > last ? last : p);
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  const u32x4 v = __builtin_nontemporal_load(reinterpret_cast<const u32x4*>(c.base + p));
  return make_uint4(v.x, v.y, v.z, v.w);
}
__device__ __forceinline__ uint4 fix16(const Corpus& c, uint64_t p, uint4 v) {
  if (p >= c.lo && p + 16 <= c.hi) return v;
  if (p + 16 <= c.lo || p >= c.hi) return make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
  uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
  for (int k = 0; k < 16; k++) {
    const uint64_t q = p + k;
    if (q < c.lo || q >= c.hi) {
      const int wi = k >> 2, sh = (k & 3) * 8;
      wv[wi] = (wv[wi] & ~(0xFFu << sh)) | (0x20u << sh);
    }
  }
  return make_uint4(wv[0], wv[1], wv[2], wv[3]);
}
__device__ __forceinline__ uint32_t nonascii16(uint4 v) { return (v.x | v.y | v.z | v.w) & 0x80808080u; }
__device__ __forceinline__ uint32_t ws_mask16(uint4 v) {
  const uint64_t l = ((uint64_t)v.y << 32) | v.x, h = ((uint64_t)v.w << 32) | v.z;
  return movemask8(ws_bytes80(l)) | (movemask8(ws_bytes80(h)) << 8);
}
__device__ __forceinline__ uint32_t zero_mask16(uint4 v) {
  const uint64_t l = ((uint64_t)v.y << 32) | v.x, h = ((uint64_t)v.w << 32) | v.z;
  return movemask8(zero_bytes80(l)) | (movemask8(zero_bytes80(h)) << 8);
}
// ASCII lowercase of 4 bytes < 0x80 (no carries between bytes), in 32-bit
// operations: the 64-bit form's constant pairs were held in SGPRs across the
// k_map row loop and spilled (a VGPR-lane reload and write-back per row)
__device__ __forceinline__ uint32_t lower4(uint32_t x) {
  // upper-case flag in bit 7 of each byte (x + 0x3F >= 0x80 and x + 0x25 < 0x80):
  // the two sums and their AND with the byte mask in one v_bitop3_b32 (5 VALU
  // instructions per dword instead of 6)
  const uint32_t up = __builtin_amdgcn_bitop3_b32(x + 0x3F3F3F3Fu, ~(x + 0x25252525u), 0x80808080u, 0x80);
  return x | (up >> 2);
}
__device__ __forceinline__ uint4 lower16(uint4 v) { return make_uint4(lower4(v.x), lower4(v.y), lower4(v.z), lower4(v.w)); }
// Whole-wave lane shifts by one on the VALU (DPP wave_shl:1 / wave_shr:1; gfx9
// family), instead of ds_bpermute through the LDS crossbar.  Lane 63 (next) and
// lane 0 (prev) get 0.
__device__ __forceinline__ uint32_t from_next_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x130, 0xF, 0xF, true);
}
__device__ __forceinline__ uint32_t from_prev_lane(uint32_t v) {
  return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x138, 0xF, 0xF, true);
}
__device__ __forceinline__ uint4 shfl_down1(uint4 v) {
  return make_uint4(__shfl_down(v.x, 1), __shfl_down(v.y, 1), __shfl_down(v.z, 1), __shfl_down(v.w, 1));
}
__device__ __forceinline__ uint4 lane0(uint4 v) {
  return make_uint4(__builtin_amdgcn_readfirstlane(v.x), __builtin_amdgcn_readfirstlane(v.y),
                    __builtin_amdgcn_readfirstlane(v.z), __builtin_amdgcn_readfirstlane(v.w));
}
// inclusive wave scan of x (wave64) on the VALU: Hillis-Steele inside each row
// of 16 lanes (DPP row_shr 1, 2, 4, 8 with zero fill), then row 0 / row 2 totals
// into the next row (row_bcast:15) and lane 31 into rows 2, 3 (row_bcast:31);
// no LDS crossbar round trips (a __shfl_up scan is 6 ds_bpermute latencies)
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x) {
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false);
  x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false);
  return x;
}

// inclusive wave max (same DPP pattern as wave_incl_scan)
__device__ __forceinline__ uint32_t wave_incl_max(uint32_t x) {
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xF, 0xF, true));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xA, 0xF, false));
  x = max(x, (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xC, 0xF, false));
  return x;
}
// v_ffbl_b32: index of the lowest set bit, ~0 for 0 (the hardware result; a
// __builtin_ctzg fallback costs a compare + select per use)
__device__ __forceinline__ uint32_t ffbl(uint32_t x) {
  uint32_t r;
  asm("v_ffbl_b32 %0, %1" : "=v"(r) : "v"(x));
  return r;
}
// LDS fetch-add issued by one lane (called under lane == 0; the result is
// lane 0's).  As inline asm because the compiler's atomic optimizer turns any
// atomic on a uniform address into a wave-aggregated one (v_mbcnt x 2, a
// compare, a bit count, two v_readfirstlane: ~8 VALU) even when one lane is
// active.  Waits for the wave's LDS operations (lgkmcnt(0)) before returning.
// a: the LDS address (a constant of the k_map layout: from a generic pointer
// the cast added a null check and SGPR spills)
__device__ __forceinline__ uint32_t lds_fetch_add1(uint32_t a, uint32_t v) {
  uint32_t r;
  asm volatile("ds_add_rtn_u32 %0, %1, %2\n\ts_waitcnt lgkmcnt(0)" : "=v"(r) : "v"(a), "v"(v) : "memory");
  return r;
}
// The same without the wait, for a compiler-managed result: the address is
// passed through a VGPR the compiler cannot see through, so it treats it as
// divergent and leaves the atomic alone (one v_mov instead of ~8 VALU).
__device__ __forceinline__ uint32_t lds_fetch_add_lane(uint32_t* p, uint32_t v) {
  uint32_t a = lds_addr(p);
  asm("" : "+v"(a));
  return atomicAdd(lds_ptr<uint32_t>(a), v);
}
// One lane's LDS add with no return value, in asm: the compiler does not count
// it in its lgkmcnt waits, which then only wait longer (LDS completes in order)
__device__ __forceinline__ void lds_add_lane(uint32_t* p, uint32_t v) {
  asm volatile("ds_add_u32 %0, %1" ::"v"(lds_addr(p)), "v"(v) : "memory");
}
#ifndef MOX_RED_LAZYCAP
#define MOX_RED_LAZYCAP 1  // k_reduce: new keys counted without a returning atomic, RED_CAP tested after the stream (-0.8 %)
#endif
// compiler + LDS ordering between lanes of one wave (LDS executes a wave's
// instructions in order; this keeps the compiler from reordering across it)
__device__ __forceinline__ void wave_lds_fence() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Token starts of a row with non-ASCII bytes (per lane, its 16 bytes): UTF-8
// validation and Unicode White_Space.  All of them take the generic walk.
__device__ uint32_t slow_starts(const MapCtx& m, uint64_t p0) {
  uint32_t st = 0;
  for (int j = 0; j < 16; j++) {
    const uint64_t p = p0 + j;
    if (p < m.c.own_lo || p >= m.c.own_hi) continue;
    const int v = utf8_check(m.c, p);
    if (v == 1) atomicMin(&rare(m).ctl->err_utf8, (unsigned long long)(p - m.c.lo));
    else if (v == 2) atomicMin(&rare(m).ctl->halo_err, (unsigned long long)(p - m.c.lo));
    if (in_ws(m.c, p)) continue;
    const bool start = (p == m.c.lo) ? true : in_ws(m.c, p - 1);
    if (start && (m.c.base[p] & 0xC0) != 0x80) st |= 1u << j;
  }
  return st;
}

// Token list entry (u16): slot offset (bits 0..9) + 1024 x length, or bit 15
// set.  An entry is odd -- a token the generic walk takes -- when it is at or
// above LIST_ODD: its length field is over 16 (the common-row list builder
// stores any length there and lets this test flag it), or bit 15 is set.
constexpr uint32_t LIST_ODD = 17u << 10;
// Key of list entry e from the lowered slot: 20 bytes read at the 4-aligned
// start, aligned and masked to len bytes by v_perm_b32 (seltab).  Split in two so
// that a token pass can issue the LDS reads of all its batches before it uses
// any of them (key_load for every batch, a scheduling barrier, then key_make):
// left alone, the scheduler waited for each batch's reads before issuing the
// next batch's, one LDS round trip per batch.  The window is read as dwords
// (ds_read2_b32 x 2 + ds_read_b32: 32-bit LDS reads take any 4-byte alignment
// without a replay), so no select between the halves of an 8-aligned window
// is needed (k_map -2.4 % against 24 bytes at the 8-aligned start).
struct KeyLd {
  uint32_t E[5];
  uint4 S;  // v_perm selectors: alignment and length mask in one (seltab)
};
// (Keys read at their exact, unaligned start and masked by AND instead of
// v_perm measured k_map +13 %: unaligned LDS reads cost far more than the four
// v_perm they save)
// List entry: slot offset in bits 0..9, length from bit 10.
__device__ __forceinline__ void key_load(const MapLds& s, const uint8_t* rowbuf, uint32_t e, KeyLd& r) {
  // rowbuf is a row slot, aligned to its size (L_ROWS): the 4-aligned token
  // offset ORs in, (e & 0x3FC) | slot in one v_bitop3_b32 (truth table 0xEA)
  const uint32_t* q = lds_ptr<const uint32_t>(__builtin_amdgcn_bitop3_b32(e, s.kmask, lds_addr(rowbuf), 0xEA));
#pragma unroll
  for (int i = 0; i < 5; i++) r.E[i] = q[i];
  // (entry 4 len + (pos & 3), as a byte offset straight from the list entry:
  // bits 6.. from len (e >> 4; nothing above it in a 16-bit entry) and bits
  // 0..5 from e << 4 (pos & 3 in bits 4..5, zero below): bit i = bit i of
  // 63 ? (e << 4) : (e >> 4), one v_bitop3_b32 with an inline constant (truth
  // table 0xD8).  An odd entry's offset may pass the table's end: it reads
  // other LDS, unused.)
  r.S = *lds_ptr<const uint4>(L_SELTAB + __builtin_amdgcn_bitop3_b32(e >> 4, e << 4, 63u, 0xD8));
}
__device__ __forceinline__ void key_make(const KeyLd& r, uint32_t (&K)[4]) {
  // byte 4 d + j of the key = byte S.d[j] of (E[d + 1]:E[d]) (0x0C: zero): one
  // v_perm_b32 per dword aligns and masks at once
  K[0] = __builtin_amdgcn_perm(r.E[1], r.E[0], r.S.x);
  K[1] = __builtin_amdgcn_perm(r.E[2], r.E[1], r.S.y);
  K[2] = __builtin_amdgcn_perm(r.E[3], r.E[2], r.S.z);
  K[3] = __builtin_amdgcn_perm(r.E[4], r.E[3], r.S.w);
}
// The rare paths of a row (byte-wise walks, Unicode checks) load from global
// memory.  Left pending where they rejoin the common path, their destination
// registers made the compiler wait for every vector memory operation in flight
// (s_waitcnt vmcnt(0)) at the next use of those registers on EVERY row, which
// in a consumer means waiting for its own cold-record stores.  Waiting at the
// end of the rare path instead keeps the common path free of that wait.
// (gfx9 encoding: vmcnt 0, expcnt 7, lgkmcnt 15)
__device__ __forceinline__ void vm_settle() { __builtin_amdgcn_s_waitcnt(0x0F70); }

// s_waitcnt immediate (gfx9 encoding) for vmcnt(v), expcnt and lgkmcnt not waited on
constexpr int vmcnt_wait(int v) { return (v & 15) | ((v >> 4) << 14) | (7 << 4) | (15 << 8); }
// the k_map loader retires its oldest row group while the LD_GROUPS - 1 younger
// groups' loads stay in flight
constexpr int LD_RETIRE_WAIT = vmcnt_wait((LD_GROUPS - 1) * LD_GROUP);
static_assert((LD_GROUPS - 1) * LD_GROUP < 64, "vmcnt is 6 bits");

// compiler scheduling barrier: no instruction moves across it
#define SCHED_FENCE() __builtin_amdgcn_sched_barrier(0)
// A sched_barrier orders only what the selection DAG left on each side of it,
// and the DAG hoists arithmetic whose operands are ready: key_make of batch 0
// landed above the fence and the mask-table reads of batches 1.. after it (one
// LDS round trip per batch).  Passing the entries through a volatile asm after
// the fence makes everything computed from them follow it.
template <int TU>
__device__ __forceinline__ void after_fence(uint32_t (&v)[TU]) {
#pragma unroll
  for (int u = 0; u < TU; u++) asm volatile("" : "+v"(v[u]));
}
#define AFTER_FENCE(v) after_fence(v)

// 16-byte key equality as one OR of XORs, each (a ^ b) | c step one
// v_bitop3_b32 (truth table 0xBE: src0 0xF0, src1 0xCC, src2 0xAA).  The
// builtin keeps the combiner from splitting it into four compares and a
// boolean tree, and (unlike inline asm, which it replaces) lets the scheduler
// interleave the chains without a wait state after every step.
// (Two v_cmp_eq_u64 per compare tied, round 5.)
__device__ __forceinline__ bool key_eq4(uint4 k, const uint32_t (&K)[4]) {
  uint32_t d = k.x ^ K[0];
  d = __builtin_amdgcn_bitop3_b32(k.y, K[1], d, 0xBE);
  d = __builtin_amdgcn_bitop3_b32(k.z, K[2], d, 0xBE);
  d = __builtin_amdgcn_bitop3_b32(k.w, K[3], d, 0xBE);
  return d == 0;
}

// Token pass over TU batches of 64 list entries (lane = token): key, hash, both
// dictionary slots' keys read at once, then an LDS count (hit) or the cold
// store (miss), so every token is decided in one LDS round trip.  All LDS reads
// of a phase are issued before the first is used (SCHED_FENCE).  The
// dictionary arrays are zero when there is no dictionary (a real key is never
// zero, so nothing hits), but that case takes pass_c.
// nvalid counts the entries taken (SALU: the valid masks' bit counts); fewer
// than the row's total means odd entries for the generic walk (do_row).
// The list is read past its last entry into the LIST_ODD tail (LIST_N; the
// batch sizes keep j < total + 64), so the reads need neither a bounds clamp
// nor an inactive-lane select.
template <int TU>
__device__ __forceinline__ void pass_a(const MapCtx& m, const uint8_t* rowbuf, const uint16_t* list, uint32_t j0,
                                       uint32_t& nvalid) {
#ifdef MOX_ISA_MARKS  // (ISA reading aid: comment markers around the token pass)
  asm volatile("; PASS_A begin TU=%0" ::"i"(TU));
#endif
  const int lane = threadIdx.x & 63;
  uint32_t e[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) e[u] = list[j0 + u * 64 + lane];
  SCHED_FENCE();  // every batch's list read in flight before the first is used
  KeyLd ld[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) key_load(m.s, rowbuf, e[u], ld[u]);
  SCHED_FENCE();
  AFTER_FENCE(e);
  uint32_t K[TU][4], h[TU], s1[TU], s2[TU];  // s1, s2: the two slots' key byte offsets (16 s)
#pragma unroll
  for (int u = 0; u < TU; u++) {
    key_make(ld[u], K[u]);
    h[u] = hash32_map(K[u][0], K[u][1], K[u][2], K[u][3]);
    s1[u] = slot_off16((h[u] & 0xFFFFu) * (uint32_t)DICT_SLOTS);  // 16 dict_s1(h)
    s2[u] = slot_off16((h[u] >> 16) * (uint32_t)DICT_SLOTS);      // 16 dict_s2(h)
  }
  // (Reading the second slot only where the first missed: fewer LDS bytes,
  // one more round trip per pass, slower; round 5.)
  uint4 d1[TU], d2[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) { d1[u] = *lds_ptr<const uint4>(L_DKEY + s1[u]); d2[u] = *lds_ptr<const uint4>(L_DKEY + s2[u]); }
  SCHED_FENCE();
  // hits count in LDS; every miss reserves its region slot (the LDS returning
  // atomics of all batches issued together), then the misses are stored
  bool miss[TU];
  uint32_t pos[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) {
    const bool valid = e[u] < LIST_ODD;
    nvalid += (uint32_t)__popcll(__ballot(valid));
    const bool hit1 = key_eq4(d1[u], K[u]), hit2 = key_eq4(d2[u], K[u]);
    miss[u] = valid & !(hit1 | hit2);
    if (valid & (hit1 | hit2) && !MOX_ABL(m.w.dbg, DBG_NO_DICTADD)) atomicAdd(lds_ptr<uint32_t>(L_DCNT + ((hit1 ? s1[u] : s2[u]) >> 2)), 1u);
#if defined(MOX_PATHS) && MOX_PATHS
    if (miss[u]) {
      if ((d1[u].x | d1[u].y | d1[u].z | d1[u].w) && hash32(d1[u].x, d1[u].y, d1[u].z, d1[u].w) == h[u]) MOX_PATH(rare(m).ctl, PATH_DICT_SAMEHASH);
      if ((d2[u].x | d2[u].y | d2[u].z | d2[u].w) && hash32(d2[u].x, d2[u].y, d2[u].z, d2[u].w) == h[u]) MOX_PATH(rare(m).ctl, PATH_DICT_SAMEHASH);
    }
#endif
  }
  if MOX_ABL(m.w.dbg, DBG_NO_COLDSTORE) return;
  // (a dictionary pass: the region counters are at L_BCNT, an immediate offset;
  // pos and bk are read under miss only.  The partition is kept opaque so
  // that it is computed once (the compiler forms the counter address from h
  // directly and shifts h again for the store): k_map +1 % without it.)
  uint32_t bk[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) {
    if (miss[u]) {
      bk[u] = bucket_of(h[u]);
      asm("" : "+v"(bk[u]));
      pos[u] = atomicAdd(lds_ptr<uint32_t>(L_BCNT + 4 * bk[u]), 1u);
    }
  }
  SCHED_FENCE();
#pragma unroll
  for (int u = 0; u < TU; u++) {
    if (!miss[u]) continue;
    const uint32_t b = bk[u];
    const uint4 key = make_uint4(K[u][0], K[u][1], K[u][2], K[u][3]);
    if (pos[u] < SPLIT_PER_REGION) note_sample(m, b, 0, pos[u], max(h[u], 1u));  // (hash32_map)
    if (pos[u] < m.rc) {
      *cold_at(m, b, 0, pos[u]) = key;
    } else {
      cold_spill(m, key);
    }
  }
#ifdef MOX_ISA_MARKS
  asm volatile("; PASS_A end");
#endif
}

// Token pass without a dictionary (high-cardinality input): every list entry
// straight to the cold path.
// (list read into its LIST_ODD tail as in pass_a; nvalid likewise)
template <int TU>
__device__ __forceinline__ void pass_c(const MapCtx& m, const uint8_t* rowbuf, const uint16_t* list, uint32_t j0,
                                       uint32_t& nvalid) {
  const int lane = threadIdx.x & 63;
  uint32_t e[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) e[u] = list[j0 + u * 64 + lane];
  SCHED_FENCE();  // every batch's list read in flight before the first is used
#pragma unroll
  for (int u = 0; u < TU; u++) nvalid += (uint32_t)__popcll(__ballot(e[u] < LIST_ODD));
  KeyLd ld[TU];
#pragma unroll
  for (int u = 0; u < TU; u++) key_load(m.s, rowbuf, e[u], ld[u]);
  SCHED_FENCE();
  AFTER_FENCE(e);
  uint32_t K[TU][4];
#pragma unroll
  for (int u = 0; u < TU; u++) key_make(ld[u], K[u]);
#pragma unroll
  for (int u = 0; u < TU; u++) {
    if (e[u] >= LIST_ODD) continue;
    const uint64_t w0 = ((uint64_t)K[u][1] << 32) | K[u][0], w1 = ((uint64_t)K[u][3] << 32) | K[u][2];
    cold_word(m, hash32_map(K[u][0], K[u][1], K[u][2], K[u][3]), w0, w1);
  }
}

// The byte flags (bit 7 of every byte) of two dwords f0, f1 into byte 3: f0's
// bytes k at bit 24 + k, f1's at 28 + k.  t holds f0's flags at 3 + 8 k and
// f1's at 7 + 8 k; copies shifted by 21 - 7 k land byte k's pair in byte 3,
// and no other flag reaches byte 3 (one v_lshrrev, one v_or, three
// v_lshl_or_b32; the former shift-right form took about 9)
__device__ __forceinline__ uint32_t gather8(uint32_t f0, uint32_t f1) {
  const uint32_t t = (f0 >> 4) | f1;
  // (as asm: left to itself the compiler folds the three into a v_mul_lo_u32 by
  // 0x204080, a quarter-rate instruction)
  uint32_t r;
  asm("v_lshl_or_b32 %0, %1, 7, %1\n\tv_lshl_or_b32 %0, %0, 7, %1\n\tv_lshl_or_b32 %0, %0, 7, %1" : "=&v"(r) : "v"(t));
  return r;
}
// the 16 byte flags of a lane's 4 dwords into bits 0..15 (bit i = byte i)
__device__ __forceinline__ uint32_t gather16(const uint32_t (&wsd)[4]) {
  return __builtin_amdgcn_perm(gather8(wsd[2], wsd[3]), gather8(wsd[0], wsd[1]), 0x0C0C0703u);
}

// per-phase cycle accounting of a map consumer wave (-DMOX_STAMP builds only)
struct Cyc {
  uint64_t wait, byte, pa, pb, miss, rows;
};

// One ring slot (64 lanes x 16 B = corpus bytes [sbase, sbase + 1024)) in two
// phases.  Lanes 1..62 hold the row's 992 payload bytes; lane 0 (the 16 bytes
// before) and lane 63 (the 16 bytes after) are context only: they give the
// previous-byte and look-ahead bits and start no token.
//  1. byte phase (lane = 16 B): token-start bit masks (SWAR on ASCII rows, the
//     Unicode walk on rows with non-ASCII bytes), the lowered slot back into LDS
//     and a compacted list of token (slot offset, length) in row order (wave
//     prefix sum of per-lane start counts from 5 bit-sliced ballots);
//  2. token phase (lane = token): pass_a over all tokens (both dictionary slots
//     read at once: an LDS count on a hit, the cold store on a miss).
__device__ __forceinline__ void do_row(const MapCtx& m, uint64_t sbase, uint4 a, unsigned long long& ntok, uint8_t* rowbuf,
                                       uint16_t* list, struct Cyc* cyc, bool edge) {
#ifdef MOX_ISA_MARKS
  asm volatile("; DO_ROW begin");
#endif
  const int lane = threadIdx.x & 63;
  const uint64_t p0 = sbase + (uint64_t)lane * 16;
  // lanes 0 and 63 are context only: their starts are cleared with a per-lane
  // mask (m.keep: a loop-invariant VGPR the compiler cannot see through; as a
  // lane-mask bool it took an SGPR pair, spilled to VGPR lanes and reloaded
  // with two v_readlane per row)
  const uint32_t keep = m.keep;
  const bool ctx = keep == 0;
  // per dword (exact for ASCII bytes: no carries between bytes): whitespace =
  // byte < 33 and (byte == 32 or 9 <= byte <= 13); control = the other bytes
  // < 33 (NUL included), flagged in bit 7 by lt33 ^ ws (ws is inside lt33 & 0x80)
  uint32_t ws16, cx = 0;
  {
    const uint32_t ad[4] = {a.x, a.y, a.z, a.w};
    uint32_t wsd[4];
    // Four adds and three v_bitop3_b32 per dword, all of the fast VALU class
    // (profiles/r05/valu_issue_probe.txt: add / bitop3 ~3 cycles, and_or / or3
    // ~5): t = (ge9 & ~ge14) | ge32 (0xBA), ws = ~ge33 & t & 0x80 (0x08),
    // control |= ~ge33 ^ ws (0xEB: (~a ^ b) | c)
#pragma unroll
    for (int d = 0; d < 4; d++) {
      const uint32_t x = ad[d];
      const uint32_t ge33 = x + 0x5F5F5F5Fu, ge32 = x + 0x60606060u, ge9 = x + 0x77777777u, ge14 = x + 0x72727272u;
      const uint32_t t = __builtin_amdgcn_bitop3_b32(ge9, ge14, ge32, 0xBA);
      wsd[d] = __builtin_amdgcn_bitop3_b32(ge33, t, 0x80808080u, 0x08);
      cx = __builtin_amdgcn_bitop3_b32(ge33, wsd[d], cx, 0xEB);
    }
    ws16 = gather16(wsd);
  }
  // one test for both rare kinds of row: a non-ASCII byte (bit 7 set; the
  // classification above is then meaningless and the row takes the Unicode
  // walk) or a control byte (NULs are found exactly below)
  bool slow = false, anyz = false;
  const uint32_t any3 = __builtin_amdgcn_bitop3_b32(a.x, a.y, a.z, 0xFE);  // (3-input ORs as bitop3: fast class)
  if (__any((__builtin_amdgcn_bitop3_b32(a.w, any3, cx, 0xFE) & 0x80808080u) != 0)) {
    slow = __any(nonascii16(a) != 0);
    anyz = !slow && __any((cx & 0x80808080u) != 0);
  }
  uint32_t ws32 = 0, z32 = 0, start;
  bool chk = false;  // rows with NUL bytes or near a non-final buffer end need the odd checks
  uint32_t lim = 64;
  if (!slow) {
    const uint32_t wsn = from_next_lane(ws16);
    const uint32_t wsp = from_prev_lane(ws16);
    ws32 = ws16 | (wsn << 16);
    start = (~ws32) & ((ws32 << 1) | ((wsp >> 15) & 1u)) & 0xFFFFu;
    start &= keep;
    if (edge && (sbase + 16 < m.c.own_lo || sbase + ROW - 16 > m.c.own_hi)) {  // edge: k_map's edge rows
      if (p0 < m.c.own_lo) start &= ~((1u << (uint32_t)(m.c.own_lo - p0 < 16 ? m.c.own_lo - p0 : 16)) - 1u);
      if (p0 + 16 > m.c.own_hi) start &= (m.c.own_hi > p0) ? ((1u << (uint32_t)(m.c.own_hi - p0)) - 1u) : 0u;
    }
    if (anyz) {
      const uint32_t z16 = zero_mask16(a);
      z32 = z16 | (from_next_lane(z16) << 16);
    }
    bool near_end = false;
    if (__builtin_expect(edge, 0)) {  // (a uniform branch: the look-ahead limit only in edge rows)
      near_end = !m.c.at_end && sbase + ROW + 32 >= m.c.hi;
      if (near_end) lim = m.c.hi > p0 ? (uint32_t)(m.c.hi - p0 < 64 ? m.c.hi - p0 : 64) : 0u;
    }
    chk = anyz || near_end;
  } else {
    start = ctx ? 0u : slow_starts(m, p0);
    vm_settle();
  }
#ifdef MOX_ISA_MARKS
  asm volatile("; MARK BP_START");
#endif
  if MOX_ABL(m.w.dbg, DBG_NO_TOKENS) { asm volatile("" ::"v"(start), "v"(z32)); return; }
  const uint32_t cnt = __popc(start);
  ntok += cnt;
  // wave-exclusive prefix of cnt (0..16) and the wave total
  const uint32_t incl = wave_incl_scan(cnt);
  const uint32_t pre = incl - cnt, total = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
  if (total == 0) return;
#ifdef MOX_ISA_MARKS
  asm volatile("; MARK BP_SCAN");
#endif
  reinterpret_cast<uint4*>(rowbuf)[lane] = lower16(a);
  // list entries: see LIST_ODD
  if (!chk && !slow) {
    // common rows: a lane's starts in order, unrolled (the entry offsets are
    // immediates) and exec-masked (a lane leaves the loop when its starts run
    // out).  The entry's fields are disjoint bits (lane base 16 lane, start
    // 0..15, length << 10): one 3-input OR (v_bitop3, fast) instead of v_add3.  A token longer than 16 bytes (or with no whitespace in the
    // window: v_ffbl of 0 is ~0) lands at or above LIST_ODD by itself and is
    // found by the token pass's valid count.
    uint32_t st = start;
    uint16_t* const mine = list + pre;  // this lane's entries: mine[0 .. cnt)
    const uint32_t lbase = (uint32_t)(lane * 16);
#ifdef MOX_ISA_MARKS
    asm volatile("; MARK LIST_PRE");
#endif
#define MOX_LIST_STEP(I)                                   \
  {                                                        \
    if (st == 0) goto list_done;                           \
    const uint32_t p = ffbl(st);                           \
    st &= st - 1;                                          \
    const uint32_t len = ffbl(ws32 >> p);                  \
    mine[I] = (uint16_t)__builtin_amdgcn_bitop3_b32(lbase, p, len << 10, 0xFE); \
  }
    MOX_LIST_STEP(0) MOX_LIST_STEP(1) MOX_LIST_STEP(2) MOX_LIST_STEP(3)
    MOX_LIST_STEP(4) MOX_LIST_STEP(5) MOX_LIST_STEP(6) MOX_LIST_STEP(7)
    MOX_LIST_STEP(8) MOX_LIST_STEP(9) MOX_LIST_STEP(10) MOX_LIST_STEP(11)
    MOX_LIST_STEP(12) MOX_LIST_STEP(13) MOX_LIST_STEP(14) MOX_LIST_STEP(15)
#undef MOX_LIST_STEP
  list_done:;
  } else {
    uint32_t k = pre;
    while (start) {
      const uint32_t p = __builtin_ctz(start);
      start &= start - 1;
      const uint32_t rest = ws32 >> p;
      const uint32_t len = rest ? __builtin_ctz(rest) : 32;
      bool odd = slow || len > 16;
      if (chk) odd = odd || p + len >= lim || ((z32 >> p) & ((1u << (len & 31)) - 1u)) != 0;
      list[k++] = (uint16_t)((uint32_t)(lane * 16) + p + (odd ? 0x8000u : (len << 10)));
    }
  }
  list[total + lane] = (uint16_t)LIST_ODD;  // the tail the token pass reads past the last entry
  wave_lds_fence();
#ifdef MOX_ISA_MARKS
  asm volatile("; DO_ROW list done");
#endif
  if MOX_ABL(m.w.dbg, DBG_NO_EMIT) { wave_lds_fence(); return; }
  uint64_t t1 = 0;
  if (cyc) { t1 = __builtin_amdgcn_s_memtime(); cyc->byte += t1; }
  uint32_t nvalid = 0;
  if (m.dict_n == 0) {  // no dictionary: no probes (uniform branch)
    for (uint32_t j0 = 0; j0 < total;) {
      if (total - j0 > 64) { pass_c<2>(m, rowbuf, list, j0, nvalid); j0 += 128; }
      else { pass_c<1>(m, rowbuf, list, j0, nvalid); j0 += 64; }
    }
  } else {
    for (uint32_t j0 = 0; j0 < total;) {
      const uint32_t rem = total - j0;
      if (rem > 128) { pass_a<3>(m, rowbuf, list, j0, nvalid); j0 += 192; }
      else if (rem > 64) { pass_a<2>(m, rowbuf, list, j0, nvalid); j0 += 128; }
      else { pass_a<1>(m, rowbuf, list, j0, nvalid); j0 += 64; }
    }
  }
  // the row has odd entries iff fewer than total were valid (tail entries are
  // not valid; uniform)
  if (nvalid != total) {
    // rare: long tokens, NUL bytes, non-ASCII rows (the order against the
    // token pass is free: every token is counted once either way)
    for (uint32_t j = lane; j < total; j += 64) {
      const uint32_t e = list[j];
      if (e >= LIST_ODD) generic_token(m, sbase + (e & 1023u));
    }
    vm_settle();
  }
  if (cyc) cyc->pa += __builtin_amdgcn_s_memtime() - t1;
  wave_lds_fence();
}


// Map kernel.  One persistent 1024-thread workgroup per CU owns a contiguous
// range of rows (992 payload bytes each).
//  * waves 0..MAP_LOADERS-1 = loaders (alternate row groups): stream each row's slot (payload +16 B either side) with
//    16 B/lane loads into registers, LD_GROUPS groups of LD_GROUP rows in
//    flight, and copies each into a free ring slot with ds_write, then
//    publishes the slot (flag written after the data by the same wave, so DS
//    ordering makes the hand-off safe).  It issues no stores to memory, so its
//    vmcnt waits are exact.
//  * the other waves = consumers: take rows in order by ticket (dynamic load
//    balance), process them from LDS (do_row) and release the slot.  Their
//    cold-record stores are never waited for inside the loop.
// resume != 0: a further launch of the same pass over the next byte range (file
// ingest overlapped with the map, mox_engine.hip run_file_overlapped): the
// region and spill counters continue from what the earlier launches wrote.
extern "C" __global__ __launch_bounds__(MAP_THREADS, MAP_MIN_WAVES) void k_map(Corpus c, Work w, uint64_t nrows, uint32_t resume) {
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  MapCtx m;
  m.c = c;
  m.w = w;
  // w's copy in the kernarg segment (k_map(Corpus, Work, ...): natural
  // alignment after c); taking &w instead would copy it to scratch
  m.wk = (KWork)((const __attribute__((address_space(4))) char*)__builtin_amdgcn_kernarg_segment_ptr() +
                 ((sizeof(Corpus) + alignof(Work) - 1) & ~(alignof(Work) - 1)));
  if (lds_addr(smem) != 0u) {  // the layout constants (L_*) assume it: never with no static LDS
    if (threadIdx.x == 0) w.ctl->layout_err = 1;
    return;
  }
  // (layout: L_ROWS ...; the per-token tables' offsets fit the LDS
  // instructions' 16-bit offset field, so no address add per access)
  m.s.dcnt = lds_ptr<uint32_t>(L_DCNT);
  m.s.bcnt = lds_ptr<uint32_t>(L_BCNT);
  m.s.misc = lds_ptr<uint32_t>(L_MISC);  // [0] spills [1] ticket
  m.s.seltab = lds_ptr<uint4>(L_SELTAB);
  m.s.dkey = lds_ptr<uint4>(L_DKEY);
  asm("v_mov_b32 %0, 0x3fc" : "=v"(m.s.kmask));
  m.keep = (uint32_t)((threadIdx.x & 63) - 1) < 62u ? 0xFFFFFFFFu : 0u;
  asm volatile("" : "+v"(m.keep));
  uint32_t* sready = lds_ptr<uint32_t>(L_RFLAGS);         // row ticket + 1 once loaded
  uint32_t* sfree = lds_ptr<uint32_t>(L_RFLAGS + RING * 4);  // row ticket + 1 once consumed
  uint8_t* ring = lds_ptr<uint8_t>(L_ROWS);
  uint16_t* lists = lds_ptr<uint16_t>(L_LISTS);
  m.s.pend = m.s.dkey;                                        // no dictionary only: dkey is all zero
  m.s.pst = reinterpret_cast<uint32_t*>(m.s.dkey + NB * QF_MAX);  // = PS_EMPTY
  static_assert(NB * QF_MAX * 16 + NB * QF_MAX * 4 <= DICT_SLOTS * 16, "pair slots inside dkey");
  static_assert(NB * QF_MAX <= DICT_SLOTS, "region counters inside dcnt");
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  m.dict_n = w.dict_hist[DH_N];
  if (MOX_ABL(w.dbg, DBG_NO_DICT)) m.dict_n = 0;
  m.qf = m.dict_n ? 1u : hc_qf(w.map_grid);
  m.qb = m.qf == 4u ? 2u : (m.qf == 2u ? 1u : 0u);
  m.rg = w.map_grid * m.qf;
  m.rc = w.cold_cap / m.qf;
  m.wcold = w.cold + (uint64_t)blockIdx.x * m.qf * NB * m.rc;
  if (!m.dict_n) m.s.bcnt = m.s.dcnt;  // NB x qf region counters
  // without a dictionary the key array is zero (no real key is zero, so nothing
  // would hit; that case takes pass_c, and the pair slots live there)
  for (int i = tid; i < DICT_SLOTS; i += MAP_THREADS) {
    m.s.dkey[i] = m.dict_n ? w.dict_key[i] : make_uint4(0, 0, 0, 0);
    m.s.dcnt[i] = 0;
  }
  __syncthreads();  // (no dictionary: the region counters live in dcnt's space)
  for (uint32_t i = tid; i < NB * m.qf; i += MAP_THREADS) {
    const uint32_t b = i >> m.qb, q = i & (m.qf - 1);
    m.s.bcnt[i] = resume ? cold_n_at(w, m.rg, blockIdx.x * m.qf + q, b) : 0u;
  }
  if (tid < 4) m.s.misc[tid] = (resume && tid == 0) ? w.spill_n[blockIdx.x] : 0u;
  if (tid < RING) { sready[tid] = 0; sfree[tid] = 0; }
  if (tid < KSEL_N) {  // key byte 4 d + j = window byte sh + 4 d + j, or 0 past len (v_perm selector 0x0C)
    const uint32_t len = (uint32_t)tid >> 2, sh = (uint32_t)tid & 3u;
    uint32_t sel[4];
#pragma unroll
    for (int d = 0; d < 4; d++) {
      sel[d] = 0;
#pragma unroll
      for (int j = 0; j < 4; j++) sel[d] |= ((uint32_t)(4 * d + j) < len ? sh + (uint32_t)j : 0x0Cu) << (8 * j);
    }
    m.s.seltab[tid] = make_uint4(sel[0], sel[1], sel[2], sel[3]);
  }
  __syncthreads();
  unsigned long long ntok = 0;

  const uint64_t base0 = c.own_lo & ~15ull;
  const uint64_t G = gridDim.x;
  const uint64_t per = nrows / G, rem = nrows % G;
  const uint64_t rb = blockIdx.x * per + (blockIdx.x < rem ? blockIdx.x : rem);
  const uint32_t n = (uint32_t)(per + (blockIdx.x < rem ? 1 : 0));

  if (wv < MAP_LOADERS) {
    // ---------------- loaders: loader wv owns row groups wv, wv + MAP_LOADERS, ...
    uint4 buf[LD_GROUPS][LD_GROUP];
    auto issue = [&](uint4 (&b)[LD_GROUP], uint32_t t0) {
#pragma unroll
      for (int i = 0; i < LD_GROUP; i++) {  // rows past n load a clamped block: uniform vmcnt counts
        const uint64_t sb = base0 + (rb + t0 + i) * PAY - 16;
        b[i] = raw16(c, sb + 16 * (uint64_t)lane);
      }
    };
    auto retire = [&](const uint4 (&b)[LD_GROUP], uint32_t t0) {
      // the whole group at once: ONE poll of its slots' free words (lane i
      // reads row t0 + i's), the rows' ds_writes back to back, then ONE store
      // publishing every row (after the data: one wave, LDS executes in
      // order).  Row by row, each row's poll waited for the previous row's
      // ds_write (lgkmcnt counts both): ~370 serial cycles per row, and the
      // loader alone took 661 us of k_map at C2 (tools/r04_ladder.sh, DBG_NO_ROW)
      // this group's loads are done once at most the younger groups' loads are
      // in flight (loads return in order).  Said explicitly, ahead of the slot
      // poll: after the poll loop the compiler's own wait was vmcnt(0), which
      // drained the loader's whole pipeline once per round of LD_GROUPS groups
      __builtin_amdgcn_s_waitcnt(LD_RETIRE_WAIT);
      {
        const uint32_t t = t0 + (uint32_t)lane;
        const bool need = lane < LD_GROUP && t < n && t >= RING;
        bool ok = !need || __hip_atomic_load(&sfree[t % RING], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == t - RING + 1;
        if (!__all(ok)) {  // (the loop only when a slot is still taken: see the wait above)
          do {
            __builtin_amdgcn_s_sleep(MOX_LD_SLEEP);
            if (!ok) ok = __hip_atomic_load(&sfree[t % RING], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == t - RING + 1;
          } while (!__all(ok));
        }
      }
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
#pragma unroll
      for (int i = 0; i < LD_GROUP; i++)
        if (t0 + i < n) reinterpret_cast<uint4*>(ring + ((t0 + i) % RING) * SLOT)[lane] = b[i];
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (lane < LD_GROUP && t0 + lane < n)
        __hip_atomic_store(&sready[(t0 + lane) % RING], t0 + lane + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    };
    __builtin_amdgcn_s_setprio(3);  // the loader feeds 15 consumers: never let it lose issue arbitration
    constexpr uint32_t STRIDE = MAP_LOADERS * LD_GROUP;  // rows between this loader's consecutive groups
    const uint32_t first = wv * LD_GROUP;
#pragma unroll
    // Groups are issued in order and each issue is fenced: the
    // retire of the oldest group then waits for that group's loads only
    // (s_waitcnt vmcnt counts loads in issue order).  Unfenced, the scheduler
    // issued the first group's loads last, so retiring it waited for every
    // load in flight: one group in flight, ~6.5 GB/s per CU, and the loader
    // alone took 661 us of k_map's ~990 at C2 (tools/r04_ladder.sh).
    for (int g = 0; g < LD_GROUPS - 1; g++) {
      issue(buf[g], first + g * STRIDE);
      SCHED_FENCE();
    }
    for (uint32_t t0 = first; t0 < n; t0 += LD_GROUPS * STRIDE) {
#pragma unroll
      for (int g = 0; g < LD_GROUPS; g++) {
        issue(buf[(g + LD_GROUPS - 1) % LD_GROUPS], t0 + (g + LD_GROUPS - 1) * STRIDE);
        SCHED_FENCE();
        retire(buf[g], t0 + g * STRIDE);
        SCHED_FENCE();
      }
    }
  } else {
    // ---------------- consumers
    uint16_t* list = lists + (wv - MAP_LOADERS) * LIST_N;
    // Edge rows: only they can reach a buffer or ownership bound.  Row r's slot
    // starts at base0 + r PAY - 16 and nrows PAY covers own_hi - base0, so every
    // row r >= 1 starts past lo and own_lo, and every row r <= nrows - 3 ends
    // ~2 rows before own_hi <= hi.  With a row of margin on each side, the other
    // rows skip the 64-bit range checks (two uniform 32-bit compares instead of
    // ~20 VALU instructions per row); a launch whose nrows does not cover its
    // range makes every row an edge row.
    uint32_t e_lo = rb < 2 ? (uint32_t)(2 - rb) : 0u;
    const uint32_t e_hi = __builtin_amdgcn_readfirstlane(nrows >= rb + 3 ? (uint32_t)min<uint64_t>(nrows - 3 - rb, n) : 0u);
    if (c.own_hi > base0 && nrows * PAY < c.own_hi - base0) e_lo = n;
#ifdef MOX_STAMP
    Cyc cyc{0, 0, 0, 0, 0, 0};
    Cyc* cp = &cyc;
#else
    Cyc* cp = nullptr;  // per-phase cycle accounting: build with -DMOX_STAMP
#endif
    for (;;) {
      const uint64_t tw = cp ? __builtin_amdgcn_s_memtime() : 0;
      uint32_t u = 0;
      if (lane == 0) u = lds_fetch_add1(L_MISC + 4, 1u);  // m.s.misc[1]
      u = __builtin_amdgcn_readfirstlane(u);
      if (u >= n) break;
      const uint32_t slot = u % RING;
      while (__hip_atomic_load(&sready[slot], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) != u + 1)
        __builtin_amdgcn_s_sleep(MOX_CO_SLEEP);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      uint8_t* sl = ring + slot * SLOT;
      const uint64_t sbase = base0 + (rb + u) * PAY - 16;
      uint4 a = reinterpret_cast<const uint4*>(sl)[lane];
      const bool edge = u < e_lo || u >= e_hi;
      if (edge && (sbase < c.lo || sbase + SLOT > c.hi)) a = fix16(c, sbase + 16 * (uint64_t)lane, a);
      if (cp) { const uint64_t t0 = __builtin_amdgcn_s_memtime(); cp->wait += t0 - tw; cp->byte -= t0; cp->rows++; }
      if (!MOX_ABL(w.dbg, DBG_NO_ROW)) do_row(m, sbase, a, ntok, sl, list, cp, edge);
      else asm volatile("" ::"v"(a.x), "v"(a.y), "v"(a.z), "v"(a.w));
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      if (lane == 0) __hip_atomic_store(&sfree[slot], u + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
    }
#ifdef MOX_STAMP
    if (lane == 0 && w.stamps) {
      unsigned long long* o = w.stamps + 8 * 4096 + ((uint64_t)blockIdx.x * MAP_WAVES + wv) * 8;
      o[0] = cyc.wait; o[1] = cyc.byte; o[2] = cyc.pa; o[3] = cyc.pb; o[4] = cyc.miss; o[5] = cyc.rows;
      o[6] = __builtin_amdgcn_s_memrealtime();  // this wave's finish (100 MHz)
    }
#endif
  }
  __syncthreads();
  if (m.dict_n == 0) {  // records still parked in pair slots: written as singles
    for (uint32_t i = tid; i < NB * m.qf; i += MAP_THREADS) {
      if (m.s.pst[i] != PS_FULL) continue;
      const uint32_t b = i >> m.qb, qr = i & (m.qf - 1);
      const uint32_t pos = atomicAdd(&m.s.bcnt[i], 1u);
      const uint4 q = m.s.pend[i];
      note_sample(m, b, qr, pos, hash32(q.x, q.y, q.z, q.w));
      if (pos < m.rc) *cold_at(m, b, qr, pos) = q;
      else cold_spill(m, q);
    }
    __syncthreads();
  }
  if (m.dict_n) {
    for (int i = tid; i < DICT_SLOTS; i += MAP_THREADS) {
      const uint32_t cnt = m.s.dcnt[i];
      if (cnt) atomicAdd(&w.dict_tot[i], (unsigned long long)cnt);
    }
  }
  // workgroup totals first: one global atomic each per workgroup (a per-thread
  // atomic on one control-block word serialises 256K updates at the L2).  They
  // live in the (now idle) token lists: k_map has no static LDS, so dynamic
  // LDS starts at address 0 and the compiler folds table bases into the LDS
  // instructions' offsets (with 16 B of static LDS it added the base per key).
  unsigned long long& s_tok = *reinterpret_cast<unsigned long long*>(lists);
  uint32_t& s_cmax = *reinterpret_cast<uint32_t*>(lists + 4);
  static_assert(MAP_LDS_BYTES % 8 == 0 && (2 * LIST_N) % 8 == 0, "totals alignment in the lists");
  if (tid == 0) { s_tok = 0; s_cmax = 0; }
  __syncthreads();
  uint32_t cmax = 0;
  for (uint32_t i = tid; i < NB * m.qf; i += MAP_THREADS) {
    const uint32_t cnt = m.s.bcnt[i], b = i >> m.qb, q = i & (m.qf - 1);
    cold_n_at(w, m.rg, blockIdx.x * m.qf + q, b) = cnt < m.rc ? cnt : m.rc;
    for (uint32_t j = cnt; j < SPLIT_PER_REGION; j++) note_sample(m, b, q, j, 0u);  // no record there (0 = none)
    cmax = cnt > cmax ? cnt : cmax;
  }
  for (int off = 32; off > 0; off >>= 1) {
    ntok += __shfl_down(ntok, off);
    const uint32_t o = __shfl_down(cmax, off);
    cmax = o > cmax ? o : cmax;
  }
  if (lane == 0) {
    if (ntok) atomicAdd(&s_tok, ntok);
    if (cmax) atomicMax(&s_cmax, cmax);
  }
  __syncthreads();
  if (tid == 0) {
    const uint32_t sn = m.s.misc[0];
    w.spill_n[blockIdx.x] = sn < w.spill_cap ? sn : w.spill_cap;
    if (sn) atomicMax(&w.ctl->spill_need, sn);
    if (s_cmax) atomicMax(&w.ctl->cold_need, (unsigned long long)s_cmax * m.qf);  // cold_cap that covers it
    if (s_tok) atomicAdd(&w.ctl->tokens, s_tok);
    if (blockIdx.x == 0) w.ctl->qf = m.qf;  // region geometry for the readers
  }
}

// Control block -> pinned host memory (device-visible): the readback of an
// async pass as a kernel, so that enqueueing it never blocks the host the way a
// small hipMemcpyAsync to host may.
extern "C" __global__ void k_ctl_out(const Ctl* __restrict__ src, Ctl* __restrict__ dst) {
  constexpr int CW = sizeof(Ctl) / 8;
  const int t = threadIdx.x;
  if (t < CW) reinterpret_cast<volatile unsigned long long*>(dst)[t] = reinterpret_cast<const unsigned long long*>(src)[t];
}

// ------------------------------------------------------------------ pass init
// One launch instead of a control-block copy and five memsets: the control
// block (zero, no UTF-8 / halo error, w_n), the partition counters, the long
// table, and (INIT_DICT) the dictionary sampling buffers or (INIT_MAP) the map
// region counters of an exchange pass.
// INIT_DICT: the dictionary is built on the pass's stream (sampling buffers
// zeroed here); INIT_DICT_SIDE: it is built on the side stream (k_dict_zero
// there), only the map's totals are zeroed; neither: no dictionary.
enum : uint32_t { INIT_DICT = 1u, INIT_MAP = 2u, INIT_DICT_SIDE = 4u };
__device__ __forceinline__ void zero_words(void* p, uint64_t bytes, uint64_t t, uint64_t stride) {
  uint4* q = reinterpret_cast<uint4*>(p);
  const uint64_t n16 = bytes / 16;
  for (uint64_t i = t; i < n16; i += stride) q[i] = make_uint4(0, 0, 0, 0);
  uint32_t* r = reinterpret_cast<uint32_t*>(q + n16);
  for (uint64_t i = t; i < (bytes % 16) / 4; i += stride) r[i] = 0;
}
extern "C" __global__ void k_init(Work w, unsigned long long w_n, uint32_t flags) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  constexpr int CW = sizeof(Ctl) / 8;
  static_assert(sizeof(Ctl) % 8 == 0, "Ctl is zeroed in 8-byte words");
  if (t < CW) {
    unsigned long long* c = reinterpret_cast<unsigned long long*>(w.ctl);
    const uint64_t off = t * 8;
    unsigned long long v = 0;
    if (off == offsetof(Ctl, err_utf8) || off == offsetof(Ctl, halo_err)) v = ~0ull;
    if (off == offsetof(Ctl, w_n)) v = w_n;
    c[t] = v;
  }
  zero_words(w.b_recs, NB * 8, t, stride);
  zero_words(w.b_w, NB * 4, t, stride);
  zero_words(w.ltab, w.long_cap * sizeof(LSlot), t, stride);
  if (flags & INIT_DICT) {
    zero_words(w.cand, (uint64_t)GC_SLOTS * sizeof(WRec), t, stride);
    zero_words(w.dict_hist, 260 * 4, t, stride);
  }
  if (flags & (INIT_DICT | INIT_DICT_SIDE)) zero_words(w.dict_tot, DICT_SLOTS * 8, t, stride);
  else if (t == 0) { w.dict_hist[DH_N] = 0; w.dict_hist[DH_T] = 0; }  // no dictionary this pass
  if (flags & INIT_MAP) {  // reduce-only pass: no map regions, no split sample
    zero_words(w.cold_n, (uint64_t)w.map_grid * NB * QF_MAX * 4, t, stride);
    zero_words(w.samp, (uint64_t)w.map_grid * NB * QF_MAX * SPLIT_PER_REGION * 4, t, stride);
    zero_words(w.spill_n, (uint64_t)w.map_grid * 4, t, stride);
  }
}

// ------------------------------------------------------------------ dictionary
// Sampling buffers of a dictionary built on the side stream (async passes):
// zeroed there, after the previous pass's k_unicode read the dictionary.
extern "C" __global__ void k_dict_zero(Work w) {
  const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (uint64_t)gridDim.x * blockDim.x;
  zero_words(w.cand, (uint64_t)GC_SLOTS * sizeof(WRec), t, stride);
  zero_words(w.dict_hist, 260 * 4, t, stride);
}
// Two-CAS claim of a 16-byte key in a global or LDS table (w1 is stored with the
// top bit set so that 0 always means "unclaimed"); used only for heuristics.
__device__ __forceinline__ bool claim16(unsigned long long* k0, unsigned long long* k1, uint64_t w0, uint64_t w1) {
  const unsigned long long t1 = w1 | (1ull << 63);
  unsigned long long o0 = atomicCAS(k0, 0ull, (unsigned long long)w0);
  if (o0 != 0 && o0 != w0) return false;
  unsigned long long o1 = atomicCAS(k1, 0ull, t1);
  return o1 == 0 || o1 == t1;
}

// ---- hot-word dictionary (heuristic: it decides speed, never counts) ----
// 1. k_sample: npieces workgroups each count the short ASCII words of one
//    SAMPLE_PIECE of the corpus (pieces spread evenly) in an LDS table and add
//    every local word into the global candidate table (cand[GC_SLOTS], claim16
//    + atomic count; one insert per distinct local word).
// 2. k_dict_hist: histogram of candidate counts (bins 0..255, 255 = >= 255).
// 3. k_dict_pick: threshold T = smallest count >= 2 with #(count >= T) <=
//    max_words; compacts those candidates into dict_list.
// 4. k_dict_build: places them hottest class first (home slot, else home
//    group, else second group) as the LDS dictionary image.
__device__ __forceinline__ uint32_t lower32(uint32_t x) {  // ASCII bytes only
  const uint32_t ge_a = x + 0x3F3F3F3Fu, gt_z = x + 0x25252525u;
  return x | (((ge_a & ~gt_z) & 0x80808080u) >> 2);
}

extern "C" __global__ __launch_bounds__(256) void k_sample(Corpus c, Work w, uint32_t npieces) {
  constexpr int BUF = SAMPLE_PIECE + 48;  // [ps - 16, ps + PIECE + 32)
  __shared__ __attribute__((aligned(16))) uint8_t buf[BUF];
  __shared__ unsigned long long sk0[SAMPLE_SLOTS], sk1[SAMPLE_SLOTS];
  __shared__ uint32_t scnt[SAMPLE_SLOTS];
  __shared__ uint4 mtab[17];
  const int tid = threadIdx.x;
  for (int i = tid; i < SAMPLE_SLOTS; i += 256) { sk0[i] = 0; sk1[i] = 0; scnt[i] = 0; }
  if (tid < 17) {
    uint32_t mk[4];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const int cc = tid - 4 * i;
      mk[i] = cc <= 0 ? 0u : (cc >= 4 ? ~0u : ((1u << (8 * cc)) - 1u));
    }
    mtab[tid] = make_uint4(mk[0], mk[1], mk[2], mk[3]);
  }
  const uint64_t span = c.own_hi - c.own_lo;
  const uint64_t stride = span / npieces;
  const uint64_t ps = (c.own_lo + stride * blockIdx.x) & ~15ull;  // 16-aligned piece start
  for (int i = tid; i < BUF / 16; i += 256) {
    const uint64_t p = ps - 16 + (uint64_t)i * 16;
    const bool in = p + 16 > c.lo && p < c.hi;
    reinterpret_cast<uint4*>(buf)[i] = in ? fix16(c, p, raw16(c, p)) : make_uint4(0x20202020u, 0x20202020u, 0x20202020u, 0x20202020u);
  }
  __syncthreads();
  // thread t: token starts in piece bytes [16 t, 16 t + 16) = buf[16 + 16 t ...]
  const uint4 own = reinterpret_cast<const uint4*>(buf)[1 + tid], nxt = reinterpret_cast<const uint4*>(buf)[2 + tid];
  const uint32_t prevb = buf[15 + 16 * tid];
  const uint32_t ws32 = ws_mask16(own) | (ws_mask16(nxt) << 16);
  uint32_t start = (~ws32) & ((ws32 << 1) | (is_ascii_ws(prevb) ? 1u : 0u)) & 0xFFFFu;
  while (start) {
    const uint32_t p = __builtin_ctz(start);
    start &= start - 1;
    const uint32_t rest = ws32 >> p;
    const uint32_t len = rest ? __builtin_ctz(rest) : 32;
    if (len > 16) continue;
    const uint32_t pos = 16 + 16 * tid + p;
    const uint2* q = reinterpret_cast<const uint2*>(buf + (pos & ~7u));
    const uint2 A = q[0], B = q[1], C = q[2];
    const uint4 M = mtab[len];
    const bool o = (pos & 4u) != 0;
    const uint32_t E0 = o ? A.y : A.x, E1 = o ? B.x : A.y, E2 = o ? B.y : B.x, E3 = o ? C.x : B.y, E4 = o ? C.y : C.x;
    const uint32_t sh = pos & 3u;
    uint32_t K[4] = {__builtin_amdgcn_alignbyte(E1, E0, sh) & M.x, __builtin_amdgcn_alignbyte(E2, E1, sh) & M.y,
                     __builtin_amdgcn_alignbyte(E3, E2, sh) & M.z, __builtin_amdgcn_alignbyte(E4, E3, sh) & M.w};
    if (((K[0] | K[1] | K[2] | K[3]) & 0x80808080u) != 0) continue;  // non-ASCII: never a dictionary word
    // zero bytes of the 16: exactly 16 - len when the token has no NUL byte
    const uint32_t nz = (uint32_t)__popcll(zero_bytes80(((uint64_t)K[1] << 32) | K[0])) +
                        (uint32_t)__popcll(zero_bytes80(((uint64_t)K[3] << 32) | K[2]));
    if (nz != 16 - len) continue;
#pragma unroll
    for (int i = 0; i < 4; i++) K[i] = lower32(K[i]);
    const uint64_t w0 = ((uint64_t)K[1] << 32) | K[0], w1 = ((uint64_t)K[3] << 32) | K[2];
    uint32_t slot = hash32(K[0], K[1], K[2], K[3]) & (SAMPLE_SLOTS - 1);
    for (int pr = 0; pr < 64; pr++) {
      if (claim16(&sk0[slot], &sk1[slot], w0, w1)) { atomicAdd(&scnt[slot], 1u); break; }
      slot = (slot + 1) & (SAMPLE_SLOTS - 1);
    }
  }
  __syncthreads();
  // compact the local words first, so that each thread runs at most a couple of
  // (dependent) global claim chains instead of one per slot it scans
  __shared__ uint16_t lw[SAMPLE_SLOTS];
  __shared__ uint32_t nlw;
  if (tid == 0) nlw = 0;
  __syncthreads();
  for (int i = tid; i < SAMPLE_SLOTS; i += 256) {
    const bool used = scnt[i] != 0 && sk0[i] != 0 && sk1[i] != 0;
    const uint64_t bm = __ballot(used);
    uint32_t b0 = 0;
    if ((tid & 63) == 0 && bm) b0 = atomicAdd(&nlw, (uint32_t)__popcll(bm));
    b0 = __shfl(b0, 0);
    if (used) lw[b0 + (uint32_t)__popcll(bm & ((1ull << (tid & 63)) - 1ull))] = (uint16_t)i;
  }
  __syncthreads();
  for (uint32_t j = tid; j < nlw; j += 256) {
    const uint32_t i = lw[j];
    const uint32_t n = scnt[i];
    const uint64_t w0 = sk0[i], w1 = sk1[i] & ~(1ull << 63);
    uint32_t g = key_hash(w0, w1) & (GC_SLOTS - 1);
    for (int pr = 0; pr < 16; pr++) {  // bounded: a full table (high-cardinality input) just drops words
      WRec* r = &w.cand[g];
      if (claim16((unsigned long long*)&r->w0, (unsigned long long*)&r->w1, w0, w1)) {
        atomicAdd((unsigned long long*)&r->count, (unsigned long long)n);
        break;
      }
      g = (g + 1) & (GC_SLOTS - 1);
    }
  }
}

extern "C" __global__ __launch_bounds__(1024) void k_dict_hist(Work w) {
  __shared__ uint32_t h[256];
  if (threadIdx.x < 256) h[threadIdx.x] = 0;
  __syncthreads();
  for (uint32_t i = blockIdx.x * 1024 + threadIdx.x; i < GC_SLOTS; i += gridDim.x * 1024) {
    const uint64_t n = w.cand[i].count;
    if (n) atomicAdd(&h[n > 255 ? 255 : n], 1u);
  }
  __syncthreads();
  if (threadIdx.x < 256 && h[threadIdx.x]) atomicAdd(&w.dict_hist[threadIdx.x], h[threadIdx.x]);
}

constexpr uint32_t DICT_MIN_COVER_INV = 20;  // a dictionary must cover >= 1/20 of the sampled tokens
extern "C" __global__ __launch_bounds__(1024) void k_dict_pick(Work w, uint32_t max_words) {
  __shared__ uint32_t T, ST, h[256];
  __shared__ unsigned long long cov[2];
  if (threadIdx.x < 256) h[threadIdx.x] = w.dict_hist[threadIdx.x];
  __syncthreads();
  // T = smallest count class cc >= 2 whose suffix sum S(cc) = sum_{c >= cc} h[c]
  // fits max_words (S is non-increasing in cc, so the fitting classes are a
  // suffix); S from an exclusive scan over the reversed histogram
  {
    __shared__ uint64_t wsum[16];
    uint64_t tot;
    const int cc = 255 - (int)threadIdx.x;
    const uint64_t x = threadIdx.x < 256 ? h[cc] : 0;
    const uint64_t ex = block_exscan(x, wsum, tot);
    if (threadIdx.x == 0) { T = 256; ST = 0; }
    __syncthreads();
    if (threadIdx.x < 254 && ex + x <= max_words) atomicMin(&T, (uint32_t)cc);  // cc in [2, 255]
    __syncthreads();
    if (threadIdx.x < 256 && cc == (int)T) ST = (uint32_t)(ex + x);  // S(T): words picked whole
    if (threadIdx.x == 0) {
      if (T > 255) T = 256;  // nothing fits: pick nothing
      cov[0] = 0;
      cov[1] = 0;
    }
    __syncthreads();
    // coverage: sampled tokens of the classes picked whole / all sampled
    // tokens.  Under DICT_MIN_COVER the dictionary would save next to nothing
    // (high-cardinality input): none is built, and k_map then sends every
    // token straight to the cold path (no probes) with paired sector writes.
    if (threadIdx.x < 256 && cc >= 1 && x) {
      const unsigned long long tok = x * (unsigned long long)cc;
      atomicAdd(&cov[0], tok);
      if ((uint32_t)cc >= T) atomicAdd(&cov[1], tok);
    }
    __syncthreads();
    if (threadIdx.x == 0) {
      if (cov[1] < cov[0] / DICT_MIN_COVER_INV) T = 256;
      if (blockIdx.x == 0) w.dict_hist[DH_T] = T;
    }
    __syncthreads();
  }
  // one slot per thread (grid = GC_SLOTS / 1024): rank picked entries in the
  // workgroup, reserve the workgroup's range with one global atomic
  // Classes >= T fill dict_list[0, S(T)) (they fit whole).  The room left
  // (max_words - S(T)) goes to class T - 1 (if >= 2) at [S(T), ...), first
  // come first served: its words are equally hot by the sample, and k_dict_build
  // places them last.
  __shared__ uint32_t wn[2][16], base[2];
  const uint32_t t = T, t1 = T - 1;
  const uint32_t i = blockIdx.x * 1024 + threadIdx.x;
  const WRec r = w.cand[i];
  const bool real = r.w0 != 0 && r.w1 != 0;
  const bool pick = real && r.count >= t;
  const bool fill = real && t1 >= 2 && t1 < 255 && r.count == t1;
  const uint64_t bm = __ballot(pick), bf = __ballot(fill);
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  if (lane == 0) { wn[0][wv] = (uint32_t)__popcll(bm); wn[1][wv] = (uint32_t)__popcll(bf); }
  __syncthreads();
  const uint64_t lt = (1ull << lane) - 1ull;
  uint32_t pre = (uint32_t)__popcll(bm & lt), pref = (uint32_t)__popcll(bf & lt), tot = 0, totf = 0;
  for (int k = 0; k < 16; k++) {
    if (k < wv) { pre += wn[0][k]; pref += wn[1][k]; }
    tot += wn[0][k];
    totf += wn[1][k];
  }
  if (threadIdx.x == 0) {
    base[0] = tot ? atomicAdd(&w.dict_hist[256], tot) : 0u;
    base[1] = totf ? atomicAdd(&w.dict_hist[257], totf) : 0u;
  }
  __syncthreads();
  if (pick) {
    const uint32_t o = base[0] + pre;
    if (o < max_words) w.dict_list[o] = WRec{r.w0, r.w1 & ~(1ull << 63), r.count};
  } else if (fill) {
    const uint32_t o = ST + base[1] + pref;
    if (o < max_words) w.dict_list[o] = WRec{r.w0, r.w1 & ~(1ull << 63), r.count};
  }
}

extern "C" __global__ __launch_bounds__(1024) void k_dict_build(Work w, uint32_t max_words) {
  __shared__ uint32_t ltag[DICT_SLOTS];
  __shared__ uint16_t lword[DICT_SLOTS];                      // word (dict_list index) in each slot
  __shared__ uint32_t klock[DICT_SLOTS / 32];                 // relocation locks, one bit per slot (one phase)
  __shared__ uint2 lk0[DICT_MAX_WORDS], lk1[DICT_MAX_WORDS];  // picked keys, staged once
  __shared__ uint8_t lcl[DICT_MAX_WORDS];                     // log2 count class
  __shared__ uint16_t order[DICT_MAX_WORDS];                  // words grouped by class, hottest first
  __shared__ uint16_t fails[DICT_MAX_WORDS];                  // words of the current class with both slots taken
  __shared__ uint32_t ccnt[32], cstart[33], cfill[32];
  __shared__ uint32_t nsel, nfail;
  const int tid = threadIdx.x;
  for (int i = tid; i < DICT_SLOTS; i += 1024) ltag[i] = 0;
  for (int i = tid; i < DICT_SLOTS / 32; i += 1024) klock[i] = 0;
  if (tid < 32) { ccnt[tid] = 0; cfill[tid] = 0; }
  if (tid == 0) nsel = 0;
  uint32_t n = w.dict_hist[256] + w.dict_hist[257];  // classes >= T, then the partial class T - 1
  if (n > max_words) n = max_words;
  __syncthreads();
  for (uint32_t i = tid; i < n; i += 1024) {
    const WRec r = w.dict_list[i];
    const uint32_t cnt = r.count > 0xFFFFFFFFull ? 0xFFFFFFFFu : (uint32_t)r.count;
    lk0[i] = make_uint2((uint32_t)r.w0, (uint32_t)(r.w0 >> 32));
    lk1[i] = make_uint2((uint32_t)r.w1, (uint32_t)(r.w1 >> 32));
    lcl[i] = (uint8_t)(31 - __clz(cnt | 1u));
    atomicAdd(&ccnt[lcl[i]], 1u);
  }
  __syncthreads();
  if (tid == 0) {  // class starts, hottest class first
    uint32_t a = 0;
    for (int cl = 31; cl >= 0; cl--) { cstart[cl] = a; a += ccnt[cl]; }
    cstart[32] = a;
  }
  __syncthreads();
  for (uint32_t i = tid; i < n; i += 1024) order[cstart[lcl[i]] + atomicAdd(&cfill[lcl[i]], 1u)] = (uint16_t)i;
  __syncthreads();
  // insert by descending log2 count class, so that a word dropped because both
  // of its slots are taken is never hotter than the words that took them.  Per
  // class: every word claims its first free slot of (s1, s2); then a word with
  // both taken tries one relocation (cuckoo step): the occupant of one of its
  // slots moves to that occupant's other slot if it is free, and the word takes
  // its place.  A slot is touched by at most one relocation per phase (klock:
  // the kicked slot and the occupant's new slot are both locked), so no
  // relocation reads a slot another one is rewriting.
  for (int cl = 31; cl >= 0; cl--) {
    const uint32_t c0 = cstart[cl], c1 = c0 + ccnt[cl];
    if (c0 == c1) continue;  // uniform
    if (tid == 0) nfail = 0;
    __syncthreads();
    for (uint32_t j = c0 + tid; j < c1; j += 1024) {
      const uint32_t i = order[j];
      const uint2 a = lk0[i], b = lk1[i];
      const uint32_t h = hash32(a.x, a.y, b.x, b.y);
      int slot = -1;
      if (atomicCAS(&ltag[dict_s1(h)], 0u, h) == 0u) slot = (int)dict_s1(h);
      else if (atomicCAS(&ltag[dict_s2(h)], 0u, h) == 0u) slot = (int)dict_s2(h);
      if (slot < 0) { fails[atomicAdd(&nfail, 1u)] = (uint16_t)i; continue; }
      lword[slot] = (uint16_t)i;
    }
    __syncthreads();
    const uint32_t nf = nfail;
    for (uint32_t j = tid; j < nf; j += 1024) {
      const uint32_t i = fails[j];
      const uint2 a = lk0[i], b = lk1[i];
      const uint32_t h = hash32(a.x, a.y, b.x, b.y);
      const uint32_t xs[2] = {dict_s1(h), dict_s2(h)};
      for (int q = 0; q < 2; q++) {
        const uint32_t x = xs[q];
        if (atomicOr(&klock[x >> 5], 1u << (x & 31)) & (1u << (x & 31))) continue;  // test-and-set
        const uint32_t ho = ltag[x];
        const uint32_t alt = dict_s1(ho) == x ? dict_s2(ho) : dict_s1(ho);
        if (alt == x) continue;
        if (atomicOr(&klock[alt >> 5], 1u << (alt & 31)) & (1u << (alt & 31))) continue;
        if (atomicCAS(&ltag[alt], 0u, ho) != 0u) continue;
        lword[alt] = lword[x];
        ltag[x] = h;
        lword[x] = (uint16_t)i;
        break;
      }
    }
    __syncthreads();
    for (int k = tid; k < DICT_SLOTS / 32; k += 1024) klock[k] = 0;
    __syncthreads();
  }
  // keys of the placed words (one writer per slot)
  for (int s2 = tid; s2 < DICT_SLOTS; s2 += 1024) {
    const uint32_t t = ltag[s2];
    uint4 key = make_uint4(0, 0, 0, 0);
    if (t) {
      const uint32_t i = lword[s2];
      key = make_uint4(lk0[i].x, lk0[i].y, lk1[i].x, lk1[i].y);
      atomicAdd(&nsel, 1u);
    }
    w.dict_key[s2] = key;
    w.dict_tag[s2] = t;
  }
  __syncthreads();
  if (tid == 0) w.dict_hist[DH_N] = nsel;  // outside the control block: a side-stream build may precede k_init
}

// Emit dictionary slot s's total (summed by k_map's atomics) as a weighted record.
__device__ __forceinline__ void dict_total(const Work& w, uint32_t s) {
  if (w.dict_hist[DH_N] == 0 || w.dict_tag[s] == 0) return;
  const uint64_t tot = w.dict_tot[s];
  if (tot == 0) return;
  const uint4 k = w.dict_key[s];
  unsigned long long i = atomicAdd(&w.ctl->w_n, 1ull);
  if (i < w.w_cap) w.w[i] = WRec{((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z, tot};
  else atomicOr(&w.ctl->overflow, OVF_W);
}

// ------------------------------------------------------------------ Unicode lane
__device__ bool t_in_ranges(uint32_t c, const uint32_t* lo, const uint32_t* hi, int n) {
  int a = 0, b = n - 1;
  while (a <= b) {
    int m = (a + b) >> 1;
    if (c < lo[m]) b = m - 1;
    else if (c > hi[m]) a = m + 1;
    else return true;
  }
  return false;
}
__device__ uint32_t t_lower(const Tables& T, uint32_t c) {
  if (c < 0x80) return (c >= 'A' && c <= 'Z') ? c + 32 : c;
  int a = 0, b = T.n_lower - 1;
  while (a <= b) {
    int m = (a + b) >> 1;
    uint32_t s = T.lower_src[m];
    if (c < s) b = m - 1;
    else if (c > s) a = m + 1;
    else return T.lower_dst[m];
  }
  return c;
}
__device__ __forceinline__ uint32_t dec_at(const uint8_t* s, uint64_t& i) {
  uint8_t c = s[i];
  if (c < 0x80) { i += 1; return c; }
  if (c < 0xE0) { uint32_t v = ((c & 0x1Fu) << 6) | (s[i + 1] & 0x3Fu); i += 2; return v; }
  if (c < 0xF0) { uint32_t v = ((c & 0x0Fu) << 12) | ((s[i + 1] & 0x3Fu) << 6) | (s[i + 2] & 0x3Fu); i += 3; return v; }
  uint32_t v = ((c & 0x07u) << 18) | ((s[i + 1] & 0x3Fu) << 12) | ((s[i + 2] & 0x3Fu) << 6) | (s[i + 3] & 0x3Fu);
  i += 4;
  return v;
}
// decode the code point that ENDS right before byte i (valid UTF-8), moving i back
__device__ __forceinline__ uint32_t dec_back(const uint8_t* s, uint64_t lo, uint64_t& i) {
  uint64_t j = i - 1;
  while (j > lo && (s[j] & 0xC0) == 0x80) j--;
  uint64_t k = j;
  uint32_t v = dec_at(s, k);
  i = j;
  return v;
}
__device__ __forceinline__ int enc_to(uint32_t cp, uint8_t* o) {
  if (cp < 0x80) { o[0] = (uint8_t)cp; return 1; }
  if (cp < 0x800) { o[0] = (uint8_t)(0xC0 | (cp >> 6)); o[1] = (uint8_t)(0x80 | (cp & 0x3F)); return 2; }
  if (cp < 0x10000) {
    o[0] = (uint8_t)(0xE0 | (cp >> 12)); o[1] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); o[2] = (uint8_t)(0x80 | (cp & 0x3F));
    return 3;
  }
  o[0] = (uint8_t)(0xF0 | (cp >> 18)); o[1] = (uint8_t)(0x80 | ((cp >> 12) & 0x3F));
  o[2] = (uint8_t)(0x80 | ((cp >> 6) & 0x3F)); o[3] = (uint8_t)(0x80 | (cp & 0x3F));
  return 4;
}

// Rust str::to_lowercase of one token (full mapping + Final_Sigma), written to
// the arena; then routed as a short key (weighted record) or a long word.
// Also emits the dictionary totals (thread s: slot s; grid >= DICT_SLOTS threads).
extern "C" __global__ void k_unicode(Corpus c, Work w, Tables T) {
  {
    const uint32_t s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s < DICT_SLOTS) dict_total(w, s);
    if (s == 0) {  // the pass's dictionary size / threshold into the control block (stats)
      w.ctl->dict_n = w.dict_hist[DH_N];
      w.ctl->dict_thresh = w.dict_hist[DH_T];
    }
  }
  if (w.ctl->err_utf8 != ~0ull) return;  // invalid input: no result is produced anyway
  uint64_t n = w.ctl->u_n;
  if (n > w.u_cap) n = w.u_cap;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n; t += (uint64_t)gridDim.x * blockDim.x) {
    URec r = w.u[t];
    const uint8_t* s = c.base;
    uint64_t cap = r.len + r.len / 2 + 4;
    unsigned long long ao = atomicAdd(&w.ctl->arena_n, (unsigned long long)cap);
    if (ao + cap > w.arena_cap) { atomicOr(&w.ctl->overflow, OVF_ARENA); continue; }
    uint8_t* out = w.arena + ao;
    uint64_t o = 0, i = r.pos, end = r.pos + r.len;
    while (i < end) {
      uint64_t at = i;
      uint32_t cp = dec_at(s, i);
      if (cp == 0x3A3) {
        // Final_Sigma (Rust map_uppercase_sigma): cased before (skipping
        // case-ignorable) and NOT (case-ignorable* cased) after, within the token.
        bool fin = false;
        uint64_t b = at;
        while (b > r.pos) {
          uint32_t pc = dec_back(s, r.pos, b);
          if (t_in_ranges(pc, T.ci_lo, T.ci_hi, T.n_ci)) continue;
          fin = t_in_ranges(pc, T.cased_lo, T.cased_hi, T.n_cased);
          break;
        }
        if (fin) {
          uint64_t f = i;
          while (f < end) {
            uint32_t nc = dec_at(s, f);
            if (t_in_ranges(nc, T.ci_lo, T.ci_hi, T.n_ci)) continue;
            if (t_in_ranges(nc, T.cased_lo, T.cased_hi, T.n_cased)) fin = false;
            break;
          }
        }
        o += enc_to(fin ? 0x3C2u : 0x3C3u, out + o);
        continue;
      }
      uint32_t l = t_lower(T, cp);
      if (l == 0x110000u) { o += enc_to(0x69u, out + o); o += enc_to(0x307u, out + o); }
      else o += enc_to(l, out + o);
    }
    bool nul = false;
    for (uint64_t k = 0; k < o; k++) nul |= (out[k] == 0);
    if (o <= 16 && !nul) {
      uint64_t w0 = 0, w1 = 0;
      for (uint64_t k = 0; k < o; k++) {
        if (k < 8) w0 |= (uint64_t)out[k] << (8 * k); else w1 |= (uint64_t)out[k] << (8 * (k - 8));
      }
      unsigned long long i2 = atomicAdd(&w.ctl->w_n, 1ull);
      if (i2 < w.w_cap) w.w[i2] = WRec{w0, w1, 1};
      else atomicOr(&w.ctl->overflow, OVF_W);
    } else {
      uint64_t h = FNV0;
      for (uint64_t k = 0; k < o; k++) h = fnv_step(h, out[k]);
      h = fnv_finish(h);
      atomicAdd(&w.ctl->long_n, 1ull);
      long_insert(w, c.base, h, ARENA_BIT | ao, o, 1);
    }
  }
}

// Partition directory (one thread per partition, NB threads): weighted and
// record offsets; run by k_hist's last workgroup.
__device__ void bucket_scan(const Work& w) {
  __shared__ uint64_t wsum[16];
  const int b = threadIdx.x;
  const uint64_t nw = ld_agent(&w.b_w[b]), nr = ld_agent((const unsigned long long*)&w.b_recs[b]);
  uint64_t sw, sr, cold;
  const uint64_t ow = block_exscan(nw, wsum, sw);
  const uint64_t orr = block_exscan(nr + nw, wsum, sr);
  (void)block_exscan(nr, wsum, cold);
  w.w_off[b] = ow;
  w.rec_off[b] = orr;
  w.b_cur[b] = 0;
  if (b == 0) {
    w.w_off[NB] = sw;
    w.rec_off[NB] = sr;
    w.ctl->cold_recs = cold;
    if (sw > w.w_cap) atomicOr(&w.ctl->overflow, OVF_W);
    if (sr > w.uniq_cap) atomicOr(&w.ctl->overflow, OVF_POOL);
    w.ctl->w_total = sw;
  }
}

// ------------------------------------------------------------------ shuffle directory
// Records per partition: cold regions (map workgroup x partition) and weighted
// records (dictionary totals, Unicode-lane words, map spills).
// Workgroup g (one per map workgroup) adds map workgroup g's region sizes and
// spills, and a grid-strided share of the weighted records.
extern "C" __global__ __launch_bounds__(1024) void k_hist(Work w) {
  __shared__ uint32_t hw[NB];
  __shared__ uint64_t hsum[16];
  const uint32_t g = blockIdx.x, G = gridDim.x;
  for (int i = threadIdx.x; i < NB; i += blockDim.x) hw[i] = 0;
  // partitions g, g + G, ...: the sum of their contiguous cold_n rows (one plain
  // agent-scope store each instead of a global atomic per (workgroup, partition))
  const uint32_t RG = reg_grid(w);  // <= MAX_MAP_GRID = blockDim (hc_qf)
  for (uint32_t b = g; b < NB; b += G) {
    uint64_t tot;
    (void)block_exscan(threadIdx.x < RG ? cold_n_at(w, RG, threadIdx.x, b) : 0u, hsum, tot);
    if (threadIdx.x == 0) st_agent((unsigned long long*)&w.b_recs[b], (unsigned long long)tot);
  }
  __syncthreads();
  uint64_t nw = w.ctl->w_n; if (nw > w.w_cap) nw = w.w_cap;
  for (uint64_t i = (uint64_t)g * blockDim.x + threadIdx.x; i < nw; i += (uint64_t)gridDim.x * blockDim.x) {
    const WRec r = w.w[i];
    atomicAdd(&hw[bucket_of(key_hash(r.w0, r.w1))], 1u);
  }
  const uint32_t ns = w.spill_n[g];
  for (uint32_t i = threadIdx.x; i < ns; i += blockDim.x) {
    const uint4 k = w.spill[(uint64_t)g * w.spill_cap + i];
    atomicAdd(&hw[bucket_of(key_hash(((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z))], 1u);
  }
  __syncthreads();
  for (int i = threadIdx.x; i < NB; i += blockDim.x)
    if (hw[i]) atomicAdd(&w.b_w[i], hw[i]);
  static_assert(NB == 1024, "k_hist's last workgroup scans one partition per thread");
  if (last_block(&w.ctl->done[0])) bucket_scan(w);
}
// Weighted records (and this map workgroup's spills) to their partition's range
// of w_sorted.  Each workgroup takes a contiguous chunk, ranks its records per
// partition in LDS, reserves one range per (workgroup, partition) with a single
// global atomic, then writes: no per-record global atomics (an exchange pass
// scatters ~1e6 received records per rank, in partition order per source).
constexpr int SCT_PER = 8;  // records per thread per sub-chunk
template <bool KEYS>  // KEYS: src holds uint4 keys (spills, count 1); else WRec
__device__ __forceinline__ void scatter_sub(const Work& w, uint32_t* lh, uint32_t* base, uint64_t n, const void* src) {
  const int tid = threadIdx.x;
  uint32_t bk[SCT_PER], li[SCT_PER];
  uint64_t r0[SCT_PER], r1[SCT_PER], rc[SCT_PER];
  for (int i = tid; i < NB; i += blockDim.x) lh[i] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SCT_PER; j++) {
    const uint64_t i = (uint64_t)j * blockDim.x + tid;
    const bool ok = i < n;
    const uint64_t ii = ok ? i : 0;
    if (KEYS) {
      const uint4 k = reinterpret_cast<const uint4*>(src)[ii];
      r0[j] = ((uint64_t)k.y << 32) | k.x;
      r1[j] = ((uint64_t)k.w << 32) | k.z;
      rc[j] = 1;
    } else {
      const WRec q = reinterpret_cast<const WRec*>(src)[ii];
      r0[j] = q.w0;
      r1[j] = q.w1;
      rc[j] = q.count;
    }
    bk[j] = ok ? bucket_of(key_hash(r0[j], r1[j])) : 0xFFFFFFFFu;
    li[j] = ok ? atomicAdd(&lh[bk[j]], 1u) : 0u;
  }
  __syncthreads();
  for (int i = tid; i < NB; i += blockDim.x) base[i] = lh[i] ? atomicAdd(&w.b_cur[i], lh[i]) : 0u;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SCT_PER; j++)
    if (bk[j] != 0xFFFFFFFFu) {
      const uint64_t q = w.w_off[bk[j]] + base[bk[j]] + li[j];
      if (MOX_CHK(w, q < w.w_off[bk[j] + 1] && q < w.w_cap, CHK_SCATTER)) w.w_sorted[q] = WRec{r0[j], r1[j], rc[j]};
    }
  __syncthreads();
}
extern "C" __global__ __launch_bounds__(1024) void k_scatter(Work w) {
  __shared__ uint32_t lh[NB], base[NB];
  if (w.ctl->w_total > w.w_cap) return;
  const uint32_t g = blockIdx.x, G = gridDim.x;
  uint64_t nw = w.ctl->w_n; if (nw > w.w_cap) nw = w.w_cap;
  const uint64_t per = (nw + G - 1) / G, lo = (uint64_t)g * per, hi = lo + per < nw ? lo + per : nw;
  const uint64_t sub = (uint64_t)SCT_PER * blockDim.x;
  for (uint64_t a = lo; a < hi; a += sub) scatter_sub<false>(w, lh, base, hi - a < sub ? hi - a : sub, w.w + a);
  const uint32_t ns = w.spill_n[g];
  const uint4* sp = w.spill + (uint64_t)g * w.spill_cap;
  for (uint64_t a = 0; a < ns; a += sub) scatter_sub<true>(w, lh, base, ns - a < sub ? ns - a : sub, sp + a);
}

// ------------------------------------------------------------------ bucket reduce
// One workgroup per partition (2 per CU): group its cold records (count 1, one
// contiguous region per map workgroup, streamed by one wave per region) and its
// weighted records by exact 16-byte key in an LDS hash table of RED_BK buckets
// x 4 slots (one ds_read_b128 of tags resolves a probe; bucket RED_BK is spare:
// only bucket RED_BK - 1 overflows into it, so a key's second bucket is always
// the next one in LDS), sort the distinct keys
// in key_less order (bucket sort + insertion sort in LDS) and write them out.  A partition with
// more distinct keys than RED_CAP is redone in 2^k sub-passes over the next
// hash bits.
// RED_BK, RED_SLOTS, RED_CAP, RED_SORTB: mox_internal.h (the host sizes the LDS)
#ifndef MOX_RED_UNROLL
#define MOX_RED_UNROLL 1  // 64-record chunks (round-4 A/B, profiles/r04/c2_k_reduce_depth_ab.txt)
#endif
constexpr int RED_UNROLL = MOX_RED_UNROLL;
#ifndef MOX_RED_DYN
#define MOX_RED_DYN 1  // k_reduce waves take chunk pairs from an LDS ticket (0: static equal shares)
#endif
#ifndef MOX_RED_TAB
#define MOX_RED_TAB 1  // k_reduce: ticket -> region table (0: binary search per ticket)
#endif
#ifndef MOX_RED_DEPTH
#define MOX_RED_DEPTH 3  // k_reduce chunks per ticket: two chunks' loads in flight while one is inserted
#endif
constexpr uint32_t RED_TICKET = 64 * MOX_RED_UNROLL * MOX_RED_DEPTH;  // records per k_reduce ticket
constexpr int RED_TAB_MAX = RED_SORTB;                  // ticket table entries (u16, in the fill space)

struct RedLds {
  uint4* tag4;             // RED_BK x 4 key hashes (0 = free)
  uint4* key;              // RED_SLOTS
  unsigned long long* cnt; // RED_SLOTS (0 = claimed, not yet published)
  uint16_t* idx;           // RED_CAP: slots in output order
  uint16_t* bin;           // RED_SORTB + 1: bin counts, then bin starts (exclusive scan)
  uint16_t* fill;          // RED_SORTB: bin fill cursors
  uint32_t* misc;          // [0] uniques [1] overflow [2] chunk ticket (MOX_RED_DYN) [3] key bytes
  uint32_t* dbg;           // DBG_COUNT: [0] slow inserts [1] slow iterations [2] publication retries
  Ctl* ctl;                // path counters (MOX_PATHS builds)
  bool plain;
};

// LDS-only workgroup barrier: the DS queue drained, no wait on global stores
// still in flight (a __syncthreads fence would wait for them).
__device__ __forceinline__ void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// hash bits used: partition = top NB_LOG2 bits, sub-pass = the next kk bits,
// bucket = a multiplicative hash of the low bits
// (fastrange of the key hash's low 16 bits: one v_mul_u32_u24 (SDWA word
// select) and a shift; the hash is already mixed, and within a partition its
// top bits are fixed while the low ones are not.  Was a 32-bit multiply by the
// golden ratio and a 24 x 10-bit product split in three instructions.)
__device__ __forceinline__ uint32_t red_bucket(uint32_t h) { return ((h & 0xFFFFu) * (uint32_t)RED_BK) >> 16; }
// (one xor and three (a ^ b) | c v_bitop3: the plain expression compiled to
// four compares, four selects and 16-bit shuffles, ~16 VALU)
__device__ __forceinline__ bool key_eq16(uint4 a, uint4 b) {
  uint32_t d = a.x ^ b.x;
  d = __builtin_amdgcn_bitop3_b32(a.y, b.y, d, 0xBE);
  d = __builtin_amdgcn_bitop3_b32(a.z, b.z, d, 0xBE);
  d = __builtin_amdgcn_bitop3_b32(a.w, b.w, d, 0xBE);
  return d == 0;
}

// Exact insert (slow path).  A slot is claimed by CAS on its tag (keys with tag
// h fill the first free slot of the first bucket with room, so every insert of
// one key walks the same buckets); the claimant then stores the key and
// publishes cnt (> 0).  Readers retry a matching slot whose cnt is still 0.
__device__ void red_insert(const RedLds& s, uint32_t h, uint4 k, uint64_t c) {
  uint32_t b = red_bucket(h);
  if (s.dbg) atomicAdd(&s.dbg[0], 1u);
  const uint32_t* tags = reinterpret_cast<const uint32_t*>(s.tag4);
  uint32_t it = 0, probes = 0, eqtag = 0;
  bool done = false;
  // wave-level loop (see long_insert): a lane that claims a slot stores the key
  // and publishes its count inside the iteration, never past the loop exit
  do {
    // a table past RED_CAP keys is redone in sub-passes anyway: stop at once
    // (a lane probing a full table would otherwise walk every bucket)
    if (!done && __hip_atomic_load(&s.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) done = true;
    if (!done) {
      const uint4 t = s.tag4[b];
      const uint32_t tv[4] = {t.x, t.y, t.z, t.w};
      bool retry = false;
#pragma unroll
      for (int i = 0; i < 4; i++) {
        if (done || retry || tv[i] != h) continue;
        const uint32_t sl = 4 * b + i;
        if (__hip_atomic_load(&s.cnt[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) == 0) { retry = true; continue; }
        __atomic_signal_fence(__ATOMIC_SEQ_CST);
        if (key_eq16(s.key[sl], k)) {
          atomicAdd(&s.cnt[sl], (unsigned long long)c);
          done = true;
        } else {
          eqtag++;  // same tag, another key (counted after the loop, as in long_insert)
        }
      }
      if (!done) {
        if (s.dbg) atomicAdd(&s.dbg[1], 1u);
        if (retry) {
          if (s.dbg) atomicAdd(&s.dbg[2], 1u);
        } else {
          // the bucket's first free slot: a bucket fills from slot 0 on and
          // slots never empty, so its taken slots are a prefix (red_try relies
          // on it)
          const int e = tv[0] == 0 ? 0 : tv[1] == 0 ? 1 : tv[2] == 0 ? 2 : tv[3] == 0 ? 3 : -1;
          if (e >= 0) {
            const uint32_t sl = 4 * b + e;
            if (atomicCAS(const_cast<uint32_t*>(&tags[sl]), 0u, h) == 0u) {
              s.key[sl] = k;
              __atomic_signal_fence(__ATOMIC_SEQ_CST);
              __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
              atomicAdd(&s.cnt[sl], (unsigned long long)c);
              const uint32_t u = atomicAdd(&s.misc[0], 1u);
              if (u >= RED_CAP) s.misc[1] = 1;
              done = true;
            }  // lost the slot: re-read this bucket
          } else {
            b = b + 1 == RED_BUCKETS ? 0 : b + 1;
            ++probes;
          }
        }
        // every bucket seen full, or (never expected) a publication that does
        // not land: the table overflows, the unit is redone in sub-passes
        if (!done && (probes >= (uint32_t)RED_BUCKETS || ++it >= 64u * RED_BUCKETS)) {
          s.misc[1] = 1;
          done = true;
        }
      }
    }
    __builtin_amdgcn_wave_barrier();
  } while (__any(!done));
  if (eqtag) MOX_PATH_ADD(s.ctl, PATH_RED_TAG, eqtag);
  (void)eqtag;
}

#ifndef MOX_RED_FASTINS
#define MOX_RED_FASTINS 1  // red_try also inserts a new key into a free slot of its first two buckets
#endif
enum : int { RED_MISS = 0, RED_ADDED = 1, RED_NEW = 2 };
// Fast path: the key's home bucket and the next one (keys overflow at most one
// bucket at this table load), their tags read together.  A bucket's taken
// slots are a prefix (red_insert), and a key sits in the first bucket that had
// room when it was inserted, so along those 8 slots the key is at the first
// slot that holds its tag or is free -- if that slot is free, the key is in
// no bucket at all and is claimed there, published in place instead of in
// red_insert's wave loop.  The slot's tag, key and count are read in one
// round trip.  RED_MISS (slow path): both buckets full without the key, a
// publication pending, a lost claim, or another key with the same tag.
__device__ __forceinline__ int red_try(const RedLds& s, uint32_t h, uint4 k, uint64_t c) {
  const uint32_t b = red_bucket(h);
  const uint4 t = s.tag4[b], t2 = s.tag4[b + 1];
  // first slot whose tag has no bit outside h: tag h or free (0), or -- about
  // 1e-4 of other tags -- a tag whose bits are a subset of h's, caught by the
  // re-read below; each select takes an inline constant
  const uint32_t nh = ~h;
  uint32_t ix = (t2.w & nh) == 0 ? 7u : 8u;
  ix = (t2.z & nh) == 0 ? 6u : ix;
  ix = (t2.y & nh) == 0 ? 5u : ix;
  ix = (t2.x & nh) == 0 ? 4u : ix;
  ix = (t.w & nh) == 0 ? 3u : ix;
  ix = (t.z & nh) == 0 ? 2u : ix;
  ix = (t.y & nh) == 0 ? 1u : ix;
  ix = (t.x & nh) == 0 ? 0u : ix;
  if (ix == 8u) {
    if (s.dbg) atomicAdd(&s.dbg[4], 1u);  // DBG_COUNT: miss reasons [4] .. [7]
    return RED_MISS;
  }
  const uint32_t sl = 4 * b + ix;
  uint32_t* tags = reinterpret_cast<uint32_t*>(s.tag4);
  // count before key (one round trip: LDS runs a wave's reads in order): a
  // published count (> 0) means the key read after it sees the key, stored
  // before the count by its claimant.  (Key first, ~275 K records per C2
  // pass read a stale key beside a fresh count and took the slow path.)
  const uint32_t tg = __hip_atomic_load(&tags[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  unsigned long long cv = __hip_atomic_load(&s.cnt[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
  __atomic_signal_fence(__ATOMIC_SEQ_CST);
  uint4 kk = s.key[sl];
  if (tg == h) {
    if (cv == 0) {  // claimed, not yet published (its claimant is a few LDS operations from it): once more
      cv = __hip_atomic_load(&s.cnt[sl], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      kk = s.key[sl];
    }
    if (cv == 0 || !key_eq16(kk, k)) {
      if (s.dbg) atomicAdd(&s.dbg[cv == 0 ? 5 : 6], 1u);
      return RED_MISS;
    }
    if (s.plain) s.cnt[sl] = cv + c;  // timing experiment only (DBG_RED_PLAINADD): loses counts
    else atomicAdd(&s.cnt[sl], (unsigned long long)c);
    return RED_ADDED;
  }
#if MOX_RED_FASTINS
  // claim: CAS from this slot on along the two buckets.  A slot lost to
  // another key moves the claim to the next slot (the slots before it are
  // taken by other keys and stay so); a slot lost to tag h was most often
  // claimed by the same key from another lane of this wave, whose claim is
  // published by the time the lane reads it -- the count is added there.
  // (At a partition's start ~1,000 lanes of 16 waves insert into the empty
  // table at once and about half of them meet in a slot.)
  for (uint32_t slc = sl;;) {
    const uint32_t prev = atomicCAS(&tags[slc], 0u, h);
    if (prev == 0u) {
      s.key[slc] = k;
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      atomicAdd(&s.cnt[slc], (unsigned long long)c);
    }
    // the wave's claims are published above before any lane reads below (LDS
    // executes a wave's instructions in order; the compiler may not move the
    // reads up into or above the branch)
    __atomic_signal_fence(__ATOMIC_SEQ_CST);
    if (prev == 0u) return RED_NEW;  // the caller counts it in misc[0]
    if (prev == h) {
      const unsigned long long c2 = __hip_atomic_load(&s.cnt[slc], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
      __atomic_signal_fence(__ATOMIC_SEQ_CST);
      const uint4 k2 = s.key[slc];
      if (c2 == 0 || !key_eq16(k2, k)) {
        if (s.dbg) atomicAdd(&s.dbg[7], 1u);
        return RED_MISS;
      }
      atomicAdd(&s.cnt[slc], (unsigned long long)c);
      return RED_ADDED;
    }
    if (++slc == 4 * b + 8) {  // both buckets full: red_insert walks on
      if (s.dbg) atomicAdd(&s.dbg[4], 1u);
      return RED_MISS;
    }
  }
#else
  return RED_MISS;
#endif
}

// Table order of short words: (h32, hash32b, key).  Every reduce kernel uses
// it (k_reduce, k_reduce_small, k_reduce_sort1), so the order does not depend
// on which kernel a key's unit went to, nor on whether its partition was split.
__device__ __forceinline__ uint32_t hash32b(uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
  // (the tie-break after h32: a different fold, multiply/xor as hash_fold's)
  uint32_t a = k1 ^ k0 * 0x2127599Bu ^ k3 * 0x165667B1u ^ k2 * 0xD3A2646Du;
  a *= 0x2C1B3C6Du;
  a ^= a >> 12;
  a *= 0x297A2D39u;
  a ^= a >> 15;
  return collide32(a, MOX_H32B_BITS);  // identity except in the collision build
}
__device__ __forceinline__ bool key_less(uint32_t ha, uint4 ka, uint32_t hb, uint4 kb) {
  if (ha != hb) return ha < hb;
  const uint32_t ga = hash32b(ka.x, ka.y, ka.z, ka.w), gb = hash32b(kb.x, kb.y, kb.z, kb.w);
  if (ga != gb) return ga < gb;
  const uint64_t a0 = ((uint64_t)ka.y << 32) | ka.x, b0 = ((uint64_t)kb.y << 32) | kb.x;
  if (a0 != b0) return a0 < b0;
  return (((uint64_t)ka.w << 32) | ka.z) < (((uint64_t)kb.w << 32) | kb.z);
}
__device__ __forceinline__ bool red_less(const RedLds& s, uint16_t a, uint16_t b) {
  if (a == 0xFFFF) return false;
  if (b == 0xFFFF) return true;
  const uint32_t* tags = reinterpret_cast<const uint32_t*>(s.tag4);
  return key_less(tags[a], s.key[a], tags[b], s.key[b]);
}

// hash bits used: partition = top NB_LOG2 bits, then (split partitions) the
// unit's sub-bucket bits, then the in-kernel sub-pass bits, then the sort bins.
// `shift` = bits above the ones being selected.
__device__ __forceinline__ uint32_t hbits(uint32_t h, uint32_t shift, uint32_t nbits) {
  if (nbits == 0 || shift >= 32) return 0;
  return (h << shift) >> (32 - nbits);
}
__device__ __forceinline__ bool in_sub(uint32_t h, uint32_t shift, uint32_t kk, uint32_t sub) {
  return kk == 0 || hbits(h, shift, kk) == sub;
}
// sort bin of a key hash: the RED_SORTB-way split of the 11 bits right below
// `shift` (ascending bin = ascending hash within the unit / sub-pass); fewer
// bits (coarser bins, still monotone) once the hash runs out.
__device__ __forceinline__ uint32_t red_bin(uint32_t h, uint32_t shift) { return shift >= 32 ? 0u : (h << shift) >> (32 - 11); }

// Every cold record of partition b (all map workgroups' regions), one wave per
// region, 4 x 64 records per chunk, the next chunk's loads in flight while the
// current one is processed (ping-pong buffers, as in k_reduce).  The wave's
// regions go in groups of 64: lane k holds the size of the group's k-th region.
template <class F>
__device__ __forceinline__ void for_cold_group(const Work& w, uint32_t b, F f, uint32_t g0, uint32_t nreg, int lane,
                                               int nwv, uint32_t RG, uint32_t RC) {
  const int wv = 0;  // regions g0 + k nwv
  const uint32_t myn = lane < (int)nreg ? cold_n_at(w, RG, g0 + lane * nwv, b) : 0u;
  const uint64_t nonempty = __ballot(myn != 0);
  auto next_region = [&](uint32_t k) -> uint32_t {  // first non-empty region index >= k
    const uint64_t m = k >= 64 ? 0ull : (nonempty >> k) << k;
    return m ? (uint32_t)__builtin_ctzll(m) : nreg;
  };
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  auto load = [&](uint32_t kq, uint32_t iq, uint4 (&v)[4]) {  // unconditional: uniform vmcnt
    const uint32_t kc = kq < nreg ? kq : 0u;
    const uint32_t n = __builtin_amdgcn_readlane(myn, kc);
    const uint4* reg = w.cold + ((uint64_t)(g0 + wv + kc * nwv) * NB + b) * RC;
#pragma unroll
    for (int u = 0; u < 4; u++) {
      const uint32_t i = iq + u * 64 + lane;
      const u32x4 x = *reinterpret_cast<const u32x4*>(reg + (i < n ? i : 0u));
      v[u] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  auto process = [&](const uint4 (&v)[4], uint32_t kq, uint32_t iq) {
    const uint32_t n = __builtin_amdgcn_readlane(myn, kq);
#pragma unroll
    for (int u = 0; u < 4; u++)
      if (iq + u * 64 + lane < n) f(v[u]);
  };
  auto advance = [&](uint32_t& kq, uint32_t& iq) {
    iq += 256;
    if (iq >= __builtin_amdgcn_readlane(myn, kq)) { kq = next_region(kq + 1); iq = 0; }
  };
  uint32_t k = next_region(0), i0 = 0;
  uint4 A[4], B[4];
  if (k < nreg) load(k, 0, A);
  while (k < nreg) {
    uint32_t kb = k, ib = i0;
    advance(kb, ib);
    load(kb, ib, B);
    process(A, k, i0);
    k = kb;
    i0 = ib;
    if (k >= nreg) break;
    uint32_t ka = k, ia = i0;
    advance(ka, ia);
    load(ka, ia, A);
    process(B, k, i0);
    k = ka;
    i0 = ia;
  }
}

template <class F>
__device__ __forceinline__ void for_partition_cold(const Work& w, uint32_t b, F f) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const uint32_t G = reg_grid(w), RC = reg_cap(w);
  const uint32_t nall = G > (uint32_t)wv ? (G - wv + nwv - 1) / nwv : 0;
  for (uint32_t r0 = 0; r0 < nall; r0 += 64)
    for_cold_group(w, b, f, wv + r0 * nwv, nall - r0 < 64 ? nall - r0 : 64u, lane, nwv, G, RC);
}

// The cold records of partition b in the regions q, q + qf, ... (slice q of
// every map workgroup: the records whose qb hash bits below the partition bits
// are q), one wave per region as in for_partition_cold.
template <class F>
__device__ __forceinline__ void for_partition_cold_q(const Work& w, uint32_t b, uint32_t q, uint32_t qf, F f) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, nwv = blockDim.x >> 6;
  const uint32_t G = reg_grid(w), RC = reg_cap(w), M = w.map_grid;
  const uint32_t nall = M > (uint32_t)wv ? (M - wv + nwv - 1) / nwv : 0;
  for (uint32_t r0 = 0; r0 < nall; r0 += 64)
    for_cold_group(w, b, f, q + qf * (wv + r0 * nwv), nall - r0 < 64 ? nall - r0 : 64u, lane, qf * nwv, G, RC);
}

// ------------------------------------------------------------------ high-cardinality split
// k_split_count (one workgroup per partition): partitions with more than
// SPLIT_MIN records estimate their distinct fraction from the first
// SPLIT_SAMPLE records (linear counting over LC_BITS hash bits).  A mostly
// distinct partition gets kk = ceil(log2(estimated distinct / SPLIT_TARGET))
// sub-bucket bits and a full histogram of its records per sub-bucket.
// Partitions with few distinct keys stay whole (their reduce resolves them in
// one table, or in a few in-kernel sub-passes).
constexpr int SC_THREADS = 256;  // 8 workgroups per CU: every partition's decision in one round
__device__ __forceinline__ void split_count(const Work& w) {
  __shared__ uint32_t bm[LC_BITS / 32];
  __shared__ uint32_t hc[SUB_N], hw[SUB_N];
  __shared__ uint64_t wsum[SC_THREADS / 64];
  __shared__ uint32_t s_ones, s_kk;
  const uint32_t b = blockIdx.x;
  const int tid = threadIdx.x;
  if (w.ctl->overflow & OVF_RERUN) { if (tid == 0) w.b_kk[b] = 0; return; }
  const uint64_t nc = w.b_recs[b], nw = w.b_w[b];
  if (nc + nw <= SPLIT_MIN) { if (tid == 0) w.b_kk[b] = 0; return; }
  for (int i = tid; i < LC_BITS / 32; i += blockDim.x) bm[i] = 0;
  if (tid == 0) s_ones = 0;
  __syncthreads();
  // sample = the first SPLIT_PER_REGION cold records of every map workgroup's
  // region (spread over the whole corpus; their key hashes, noted by k_map),
  // topped up with weighted records
  const uint32_t G = reg_grid(w), QF = reg_qf(w), MG = G / QF;
  // sample slot rj (of NS = 256) reads region QF g + q of map workgroup g =
  // rj MG / NS (spread evenly over all map workgroups, so over the whole
  // corpus) with q = rj mod QF rotating through the slices; a grid of at most
  // NS regions is sampled whole
  constexpr uint32_t NS = SPLIT_SAMPLE / SPLIT_PER_REGION;
  auto mark = [&](uint32_t h) {
    const uint32_t bit = hbits(h, NB_LOG2, 12);  // LC_BITS = 2^12
    atomicOr(&bm[bit >> 5], 1u << (bit & 31));
  };
  uint32_t mine = 0;
  {
    constexpr int PER = (SPLIT_SAMPLE + SC_THREADS - 1) / SC_THREADS;  // sample slots per thread
    uint32_t v[PER];
#pragma unroll
    for (int j = 0; j < PER; j++) {  // k_map's note_sample: contiguous per partition, 0 = no record
      const uint32_t idx = tid + j * SC_THREADS;
      const uint32_t rj = idx / SPLIT_PER_REGION;
      const uint32_t reg = G <= NS ? rj : (uint32_t)((uint64_t)rj * MG / NS) * QF + rj % QF;
      v[j] = idx < SPLIT_SAMPLE && reg < G ? w.samp[((uint64_t)b * G + reg) * SPLIT_PER_REGION + idx % SPLIT_PER_REGION] : 0u;
    }
#pragma unroll
    for (int j = 0; j < PER; j++)
      if (v[j]) { mark(v[j]); mine++; }
  }
  uint64_t cs;
  (void)block_exscan(mine, wsum, cs);
  const uint64_t ws = cs < SPLIT_SAMPLE ? (nw < SPLIT_SAMPLE - cs ? nw : SPLIT_SAMPLE - cs) : 0;
  const uint64_t w0 = w.w_off[b];
  for (uint64_t i = tid; i < ws; i += blockDim.x) { const WRec r = w.w_sorted[w0 + i]; mark(key_hash(r.w0, r.w1)); }
  __syncthreads();
  for (int i = tid; i < LC_BITS / 32; i += blockDim.x) atomicAdd(&s_ones, (uint32_t)__popc(bm[i]));
  __syncthreads();
  if (tid == 0) {
    const float n_s = (float)(cs + ws);
    const float zeros = (float)(LC_BITS - s_ones);
    const float d = zeros > 0.f ? -(float)LC_BITS * __logf(zeros / (float)LC_BITS) : n_s;
    const float r = n_s > 0.f ? fminf(d / n_s, 1.f) : 0.f;
    uint32_t kk = 0;
    if (r >= 0.5f) {
      const float est = (float)(nc + nw) * r;
      while (kk < SUB_BITS_MAX && est > (float)SPLIT_TARGET * (float)(1u << kk)) kk++;
    }
    s_kk = kk;
    w.b_kk[b] = kk;
  }
  __syncthreads();
  const uint32_t kk = s_kk;
  if (!kk) return;
  const uint32_t nsub = 1u << kk;
  for (uint32_t i = tid; i < nsub; i += blockDim.x) { hc[i] = 0; hw[i] = 0; }
  __syncthreads();
  for_partition_cold(w, b, [&](uint4 k) { atomicAdd(&hc[hbits(hash32(k.x, k.y, k.z, k.w), NB_LOG2, kk)], 1u); });
  for (uint64_t i = w0 + tid; i < w0 + nw; i += blockDim.x) {
    const WRec r = w.w_sorted[i];
    atomicAdd(&hw[hbits(key_hash(r.w0, r.w1), NB_LOG2, kk)], 1u);
  }
  __syncthreads();
  uint32_t* o = w.sub_hist + (uint64_t)b * 2 * SUB_N;
  for (uint32_t i = tid; i < nsub; i += blockDim.x) { o[i] = hc[i]; o[SUB_N + i] = hw[i]; }
}

// split_k records reserved for a split partition of n cold records in 2^kk
// sub-buckets: every sub-bucket starts at an even record (32-byte aligned) so
// that k_split_scatter's record pairs fill whole 32-byte sectors; even total.
__device__ __forceinline__ uint64_t split_span(uint64_t n, uint32_t kk) { return (n + (1ull << kk) + 1) & ~1ull; }

// One workgroup of SC_THREADS threads, SC_PER consecutive partitions each:
// units per partition, split-buffer offsets, the reduce work-queue reset, and
// the output region of every whole partition.
constexpr int SC_PER = NB / SC_THREADS;
constexpr int SC_BINS = 256;  // size classes of the k_reduce order (one per thread)
static_assert(SC_BINS == SC_THREADS && SC_PER * SC_THREADS == NB, "k_unit_scan geometry");
__device__ void unit_scan(const Work& w) {
  __shared__ uint64_t wsum[16];
  __shared__ uint32_t smax, smin, bins[SC_BINS], fill[SC_BINS];
  const int t = threadIdx.x;
  uint32_t kk[SC_PER], sz[SC_PER];
  uint64_t nu = 0, nk = 0, nw = 0, nwh = 0;
  if (t == 0) { smax = 0; smin = 0xFFFFFFFFu; }
  bins[t] = 0;
  fill[t] = 0;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SC_PER; j++) {
    const uint32_t b = SC_PER * t + j;
    kk[j] = w.b_kk[b];
    const uint64_t nr = w.b_recs[b], nwb = w.b_w[b];
    sz[j] = kk[j] ? 0u : (uint32_t)min(nr + nwb, 0x7FFFFFFFull);  // split partitions: their units go to the queues
    nu += 1ull << kk[j];
    nk += kk[j] ? split_span(nr, kk[j]) : 0;
    nw += kk[j] ? nwb : 0;
    nwh += kk[j] ? 0 : 1;
  }
  {  // size range of the whole partitions: wave max / min on the VALU, one LDS atomic per wave
    uint32_t mx = 0, mn = 0xFFFFFFFFu;
#pragma unroll
    for (int j = 0; j < SC_PER; j++) {
      mx = max(mx, sz[j]);
      mn = kk[j] ? mn : min(mn, sz[j]);
    }
    mx = (uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(mx), 63);
    mn = ~(uint32_t)__builtin_amdgcn_readlane((int)wave_incl_max(~mn), 63);
    if ((t & 63) == 0) { atomicMax(&smax, mx); atomicMin(&smin, mn); }
  }
  // k_reduce order: whole partitions by descending size class (workgroup i of
  // k_reduce takes red_order[i]; the first resident round gets the biggest, the
  // second the smallest: the two rounds balance instead of a big partition
  // starting late), split partitions last (their workgroups go straight to the
  // work queue)
  __syncthreads();
  const uint32_t lo = smin <= smax ? smin : 0u, span = smax - lo + 1;  // sizes of whole partitions spread over the bins
  uint32_t bin[SC_PER];
#pragma unroll
  for (int j = 0; j < SC_PER; j++) {
    const uint32_t r = kk[j] ? 0u : sz[j] - lo;  // split partitions: smallest class (their workgroups take queued units)
    bin[j] = SC_BINS - 1 - (uint32_t)(((uint64_t)r * SC_BINS) / span);  // 0 = biggest
    atomicAdd(&bins[bin[j]], 1u);
  }
  __syncthreads();
  {
    uint64_t tot;
    const uint32_t c = bins[t];
    const uint32_t ex = (uint32_t)block_exscan(c, wsum, tot);
    bins[t] = ex;
  }
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SC_PER; j++) w.red_order[bins[bin[j]] + atomicAdd(&fill[bin[j]], 1u)] = SC_PER * t + j;
  uint64_t U, tk, tw, nwhole;
  uint64_t ub = block_exscan(nu, wsum, U);
  uint64_t ok = block_exscan(nk, wsum, tk);
  uint64_t ow = block_exscan(nw, wsum, tw);
  (void)block_exscan(nwh, wsum, nwhole);
#pragma unroll
  for (int j = 0; j < SC_PER; j++) {
    const uint32_t b = SC_PER * t + j;
    w.u_base[b] = (uint32_t)ub;
    w.b_uniq[b] = 0;  // k_reduce*: set (whole partition) or accumulated (split)
    w.sp_off[b] = ok;
    w.spw_off[b] = ow;
    if (!kk[j]) w.udesc[ub] = UnitDesc{0, 0, w.rec_off[b], UNIT_WHOLE, 0, b, 0};
    ub += 1ull << kk[j];
    ok += kk[j] ? split_span(w.b_recs[b], kk[j]) : 0;
    ow += kk[j] ? w.b_w[b] : 0;
  }
  if (t == 0) {
    w.u_base[NB] = (uint32_t)U;
    w.sp_off[NB] = tk;
    w.spw_off[NB] = tw;
    w.ctl->n_units = U;
    w.ctl->n_big = 0;  // k_split_scatter lists oversized sub-buckets (whole partitions: k_reduce workgroup b)
    w.ctl->n_mid = 0;  // ... and the count-1 ones of up to 2 SMALL_CAP records (k_reduce_sort2)
    w.ctl->n_small = 0;  // ... and the small ones with weighted records (k_reduce_small)
    w.ctl->red_ticket = 0;
    w.ctl->split_k = tk;
    w.ctl->split_w = tw;
    w.ctl->n_split = (uint32_t)(NB - nwhole);
    if (tk > w.split_k_cap || tw > w.split_w_cap) atomicOr(&w.ctl->overflow, OVF_SPLIT);
  }
}
extern "C" __global__ __launch_bounds__(SC_THREADS) void k_split_count(Work w) { split_count(w); }
extern "C" __global__ __launch_bounds__(SC_THREADS) void k_unit_scan(Work w) { unit_scan(w); }  // one workgroup

// k_split_scatter (one workgroup per split partition): unit directory from the
// histogram, then every record of the partition to its unit's contiguous range
// (LDS cursors: the workgroup owns the whole partition, no global atomics).
// Records are written in pairs: a sub-bucket's first record waits in an LDS
// slot until the next one arrives, and the pair goes out as one aligned
// 32-byte sector (a lone 16-byte store leaves half a sector, which costs the
// memory a read-modify-write: PMC WRITE_SIZE was 2x the records).  The slot is
// a three-state LDS lock (EMPTY / BUSY / FULL): a lane that finds it BUSY
// retries, and the BUSY holder finishes within the same loop iteration, so no
// lane ever waits on another wave's progress.  Leftover single records are
// written after the stream.
#ifndef MOX_SPLIT_STAGE
#define MOX_SPLIT_STAGE 1  // slices of QF-region partitions go out LDS-staged (0: record pairs, the round-3 scheme)
#endif
// LDS-staged scatter of slice q (regions q, q + qf, ...) of partition b: the
// slice's records in chunks of SST_CH, each chunk counting-sorted by sub-bucket
// in LDS, then every sub-bucket's run of the chunk written with consecutive
// stores (a slice opens nsub / qf sub-buckets: ~6 records, 96 B, per run at
// C4 16 GiB instead of one 32-byte pair per store).
constexpr int SST_CH = 6144;
constexpr int SST_PER = SST_CH / 1024;
struct SplitStage {
  uint4* stage;      // SST_CH records of the chunk, by sub-bucket
  uint16_t* sidx;    // SST_CH: each staged record's sub-bucket (slice-local)
  uint32_t* lcnt;    // 1024: the chunk's records per slice-local sub-bucket
  uint32_t* lst;     // 1024: their first stage position
  uint32_t* gb;      // 1024: their first output record (split_k, partition-relative)
  uint32_t* rpre;    // MAX_MAP_GRID + 1: prefix of the slice's region sizes
};
__device__ void split_stage_slice(const Work& w, uint32_t b, uint32_t q, uint32_t qf, uint32_t kk, uint32_t* cc, uint4* ok,
                                  uint64_t tc, uint64_t kb, const SplitStage& S, uint64_t* wsum) {
  const int tid = threadIdx.x;
  const uint32_t G = reg_grid(w), RC = reg_cap(w), M = w.map_grid;
  const uint32_t qb = qf == 4u ? 2u : 1u, F = (1u << kk) >> qb, sb0 = q * F;
  {
    uint64_t tot;
    const uint32_t n = tid < (int)M ? cold_n_at(w, G, q + qf * tid, b) : 0u;
    const uint64_t ex = block_exscan(n, wsum, tot);
    if (tid < (int)M) S.rpre[tid] = (uint32_t)ex;
    if (tid == 0) S.rpre[M] = (uint32_t)tot;
    if (tid < (int)F) S.lcnt[tid] = 0;
  }
  __syncthreads();
  const uint32_t n = S.rpre[M];
  uint32_t r = 0, rs = 0, re = S.rpre[1];  // this thread's region walk (its indices only grow)
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  // the chunk's records; the next chunk's loads are issued as soon as these
  // are in the stage, so they are in flight during this chunk's stores (the
  // stores are a fixed count of predicated instructions: waiting for the
  // loads then needs vmcnt(SST_PER), not vmcnt(0) behind the stores)
  uint4 k[SST_PER];
  auto load_chunk = [&](uint32_t c0) {
#pragma unroll
    for (int j = 0; j < SST_PER; j++) {
      const uint32_t i = c0 + j * 1024 + tid;
      const bool ok_i = i < n;
      while (ok_i && i >= re) { r++; rs = re; re = S.rpre[r + 1]; }
      const uint4* p = w.cold + ((uint64_t)(q + qf * r) * NB + b) * RC + (ok_i ? i - rs : 0u);
      const u32x4 x = *reinterpret_cast<const u32x4*>(ok_i ? p : w.cold);
      k[j] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  if (n) load_chunk(0);
  for (uint32_t c0 = 0; c0 < n; c0 += SST_CH) {
    uint32_t sub[SST_PER], rk[SST_PER];
#pragma unroll
    for (int j = 0; j < SST_PER; j++) {
      const uint32_t i = c0 + j * 1024 + tid;
      sub[j] = i < n ? hbits(hash32(k[j].x, k[j].y, k[j].z, k[j].w), NB_LOG2, kk) - sb0 : 0xFFFFu;
      rk[j] = i < n ? atomicAdd(&S.lcnt[sub[j]], 1u) : 0u;
    }
    __syncthreads();
    {  // slice-local sub-bucket starts in the stage; their output cursors advance
      uint64_t tot;
      const uint32_t cnt = tid < (int)F ? S.lcnt[tid] : 0u;
      const uint32_t ex = (uint32_t)block_exscan(cnt, wsum, tot);
      if (tid < (int)F) {
        S.lst[tid] = ex;
        S.gb[tid] = cc[sb0 + tid];
        cc[sb0 + tid] += cnt;
        S.lcnt[tid] = 0;
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < SST_PER; j++)
      if (sub[j] != 0xFFFFu) {
        const uint32_t pos = S.lst[sub[j]] + rk[j];
        S.stage[pos] = k[j];
        S.sidx[pos] = (uint16_t)sub[j];
      }
    if (c0 + SST_CH < n) load_chunk(c0 + SST_CH);
    __syncthreads();
    const uint32_t nc = n - c0 < (uint32_t)SST_CH ? n - c0 : (uint32_t)SST_CH;
#pragma unroll
    for (int jj = 0; jj < SST_PER; jj++) {
      const uint32_t j = tid + jj * 1024;
      if (j < nc) {
        const uint32_t sb = S.sidx[j];
        const uint32_t d = S.gb[sb] + (j - S.lst[sb]);
        if (MOX_CHK(w, d < tc && kb + d < w.split_k_cap, CHK_SPLIT_K)) ok[d] = S.stage[j];
      }
    }
    lds_barrier();  // the stage is rewritten by the next chunk (LDS only: the stores need not land first)
  }
}

extern "C" __global__ __launch_bounds__(1024) void k_split_scatter(Work w) {
  __shared__ uint32_t cc[SUB_N], cw[SUB_N];
  // pair slots, or (staged slices) the stage: one LDS area
  constexpr int PAIR_B = SUB_N * 4 + SUB_N * 16;
  constexpr int STAGE_B = SST_CH * 16 + SST_CH * 2 + 3 * 1024 * 4 + (MAX_MAP_GRID + 4) * 4;
  __shared__ __attribute__((aligned(16))) uint8_t xs[PAIR_B > STAGE_B ? PAIR_B : STAGE_B];
  uint32_t* pst = reinterpret_cast<uint32_t*>(xs);
  uint4* pend = reinterpret_cast<uint4*>(xs + SUB_N * 4);
  __shared__ uint64_t wsum[16];
  const uint32_t b = blockIdx.x;
  const int tid = threadIdx.x;
  const uint32_t kk = w.b_kk[b];
  if (!kk || (w.ctl->overflow & OVF_RERUN)) return;
  const uint32_t nsub = 1u << kk, u0 = w.u_base[b];
  const uint32_t* hist = w.sub_hist + (uint64_t)b * 2 * SUB_N;
  // sub-buckets SUB_PER_T t .. SUB_PER_T t + SUB_PER_T - 1 per thread
  uint32_t c[SUB_PER_T], d[SUB_PER_T], sc = 0, sd = 0, sr = 0;
#pragma unroll
  for (int j = 0; j < SUB_PER_T; j++) {
    const uint32_t sb = SUB_PER_T * tid + j;
    c[j] = sb < nsub ? hist[sb] : 0;
    d[j] = sb < nsub ? hist[SUB_N + sb] : 0;
    sc += (c[j] + 1) & ~1u;  // split_k: even starts
    sd += d[j];
    sr += c[j];              // output region: records, no padding
  }
  __shared__ uint32_t ncat[4];
  __shared__ unsigned long long gcat[4];
  if (tid < 4) ncat[tid] = 0;  // (ordered before the adds below by block_exscan's barriers)
  uint64_t tc, tw, tr;
  uint64_t ec = block_exscan(sc, wsum, tc);
  uint64_t ew = block_exscan(sd, wsum, tw);
  uint64_t er = block_exscan(sr, wsum, tr);
  const uint64_t kb = w.sp_off[b], wb = w.spw_off[b], rb = w.rec_off[b];
  // work lists of the unit kernels: each unit's rank inside this workgroup's
  // share of its list (LDS), then one global add per list and workgroup (the
  // lists' order is free: units are placed by their descriptors)
  uint32_t cat[SUB_PER_T], lr[SUB_PER_T];
#pragma unroll
  for (int j = 0; j < SUB_PER_T; j++) {
    const uint32_t sb = SUB_PER_T * tid + j;
    cat[j] = 3;  // none
    if (sb < nsub) {
      const uint32_t u = u0 + sb;
      if (MOX_CHK(w, u < U_MAX, CHK_UNIT)) w.udesc[u] = UnitDesc{kb + ec, wb + ew, rb + er + ew, c[j], d[j], b, kk};
      if (d[j] == 0 && c[j] > SMALL_CAP && c[j] <= 2 * SMALL_CAP) cat[j] = 0;  // count-1, up to twice sort1's size: k_reduce_sort2
      else if (c[j] + d[j] > SMALL_CAP) cat[j] = 1;                            // k_reduce
      else if (d[j] != 0) cat[j] = 2;  // weighted records, <= SMALL_CAP in all: k_reduce_small
      if (cat[j] < 3) lr[j] = atomicAdd(&ncat[cat[j]], 1u);
      cc[sb] = (uint32_t)ec;
      cw[sb] = (uint32_t)ew;
      pst[sb] = PS_EMPTY;
    }
    ec += (c[j] + 1) & ~1u;
    ew += d[j];
    er += c[j];
  }
  __syncthreads();
  if (tid < 3 && ncat[tid]) gcat[tid] = atomicAdd(tid == 0 ? &w.ctl->n_mid : tid == 1 ? &w.ctl->n_big : &w.ctl->n_small,
                                                  (unsigned long long)ncat[tid]);
  __syncthreads();
#pragma unroll
  for (int j = 0; j < SUB_PER_T; j++)
    if (cat[j] < 3) {
      const unsigned long long q = gcat[cat[j]] + lr[j];
      uint32_t* list = cat[j] == 0 ? w.mid_units : cat[j] == 1 ? w.big_units : w.small_units;
      if (MOX_CHK(w, q < U_MAX, CHK_UNIT)) list[q] = u0 + SUB_PER_T * tid + j;
    }
  uint4* ok = w.split_k + kb;
  // (the lambda runs under a per-record lane mask; the pair loop is the same
  // wave-level loop as k_map's cold_pair)
  auto put = [&](uint4 k) {
    const uint32_t sb = hbits(hash32(k.x, k.y, k.z, k.w), NB_LOG2, kk);
    bool done = false;
    do {
      if (!done) {
        uint4 q;
        const int r = pair_try(pst, pend, sb, k, &q);
        if (r == 2) {  // second of a pair: the pair goes out as one sector
          const uint32_t p = atomicAdd(&cc[sb], 2u);
          if (MOX_CHK(w, p + 1 < tc && kb + p + 1 < w.split_k_cap, CHK_SPLIT_K)) {
            ok[p] = q;
            ok[p + 1] = k;
          }
        }
        done = r != 0;
      }
      __builtin_amdgcn_wave_barrier();
    } while (__any(!done));
  };
  // slice by slice (k_map without a dictionary keeps qf slices per region, by
  // the hash bits right below the partition bits = the top sub-bucket bits): a
  // slice's records go to a qf-th of the sub-buckets, so fewer output lines are
  // open at once
  const uint32_t qf = reg_qf(w);
  const bool sliced = qf > 1 && kk >= (qf == 4u ? 2u : 1u);
  // the stage's per-sub-bucket arrays (lcnt, lst, gb) hold 1,024 entries: a
  // slice opens (2^kk) / qf sub-buckets, which exceeds that only for qf = 2 and
  // kk = 12 (a 257..512-workgroup map grid); such a slice takes the pair path
  const bool stage_fits = ((1u << kk) >> (qf == 4u ? 2u : 1u)) <= 1024u;
  if (w.b_recs[b] == 0) {
    // no cold records (the exchange's and mox_reduce_pairs' reduce passes):
    // only the weighted records below
  } else if (sliced && stage_fits && MOX_SPLIT_STAGE) {
    SplitStage S;
    S.stage = reinterpret_cast<uint4*>(xs);
    S.sidx = reinterpret_cast<uint16_t*>(xs + SST_CH * 16);
    S.lcnt = reinterpret_cast<uint32_t*>(xs + SST_CH * 18);
    S.lst = S.lcnt + 1024;
    S.gb = S.lst + 1024;
    S.rpre = S.gb + 1024;
    for (uint32_t q = 0; q < qf; q++) split_stage_slice(w, b, q, qf, kk, cc, ok, tc, kb, S, wsum);
  } else if (sliced) {
    for (uint32_t q = 0; q < qf; q++) {
      for_partition_cold_q(w, b, q, qf, put);
      __syncthreads();
    }
  } else {
    for_partition_cold(w, b, put);
  }
  const uint64_t w0 = w.w_off[b], w1 = w.w_off[b + 1];
  WRec* ow = w.split_w + wb;
  constexpr int WB = 4;  // weighted records per thread and round, all loads issued before the first is used
  for (uint64_t i0 = w0 + tid; i0 < w1; i0 += WB * blockDim.x) {
    WRec r[WB];
#pragma unroll
    for (int q = 0; q < WB; q++) {
      const uint64_t i = i0 + (uint64_t)q * blockDim.x;
      if (i < w1) r[q] = w.w_sorted[i];
    }
#pragma unroll
    for (int q = 0; q < WB; q++)
      if (i0 + (uint64_t)q * blockDim.x < w1) {
        const uint32_t p = atomicAdd(&cw[hbits(key_hash(r[q].w0, r[q].w1), NB_LOG2, kk)], 1u);
        if (MOX_CHK(w, p < tw && wb + p < w.split_w_cap, CHK_SPLIT_W)) ow[p] = r[q];
      }
  }
  __syncthreads();
  if (sliced && MOX_SPLIT_STAGE) return;  // (no pair slots)
  // leftover singles (odd counts)
#pragma unroll
  for (int j = 0; j < SUB_PER_T; j++) {
    const uint32_t sb = SUB_PER_T * tid + j;
    if (sb < nsub && pst[sb] == PS_FULL) {
      const uint32_t p = cc[sb];
      if (MOX_CHK(w, p < tc && kb + p < w.split_k_cap, CHK_SPLIT_K)) ok[p] = pend[sb];
    }
  }
}

// ------------------------------------------------------------------ unit reduce
// Persistent workgroups (2 per CU) take reduce units from a work queue.  A unit
// is a whole partition (its cold regions + its weighted records) or one
// sub-bucket of a split partition (contiguous ranges of split_k / split_w).
extern "C" __global__ __launch_bounds__(RED_THREADS, 8) void k_reduce(Work w) {  // 8 waves per SIMD: 2 workgroups per CU
  extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
  RedLds s;
  uint8_t* sp = smem;
  s.tag4 = (uint4*)sp; sp += RED_SLOTS * 4;
  s.key = (uint4*)sp; sp += RED_SLOTS * 16;
  s.cnt = (unsigned long long*)sp; sp += RED_SLOTS * 8;
  s.idx = (uint16_t*)sp; sp += RED_CAP * 2;
  s.bin = (uint16_t*)sp; sp += (RED_SORTB + 8) * 2;
  s.fill = (uint16_t*)sp; sp += RED_SORTB * 2;
  s.misc = (uint32_t*)sp; sp += 16;
  __shared__ uint32_t dbgc[8];
  __shared__ uint32_t s_unit;
  __shared__ uint64_t red_wsum[RED_THREADS / 64];
  uint32_t* rpre = reinterpret_cast<uint32_t*>(s.idx);  // region prefix (G + 1 words in the idx + bin space)
  uint16_t* rtab = s.fill;                              // ticket -> region (fill space: free until the sort)
  static_assert(RED_CAP * 2 + (RED_SORTB + 8) * 2 >= (MAX_MAP_GRID + 1) * 4, "region prefix space");
  s.dbg = MOX_ABL(w.dbg, DBG_COUNT) ? dbgc : nullptr;
  s.plain = MOX_ABL(w.dbg, DBG_RED_PLAINADD) != 0;
  s.ctl = w.ctl;
  if (threadIdx.x < 8) dbgc[threadIdx.x] = 0;
  const int tid = threadIdx.x, lane = tid & 63;
  [[maybe_unused]] const int wv = tid >> 6;
  [[maybe_unused]] constexpr int NWV = RED_THREADS / 64;
  const uint32_t G = reg_grid(w), RC = reg_cap(w);  // cold regions per partition (<= MAX_MAP_GRID), records per region
  uint32_t* tags = reinterpret_cast<uint32_t*>(s.tag4);
  // an overflowed map, directory or split means this attempt is rerun with
  // larger buffers: its records are incomplete (nothing downstream reads them)
  if (w.ctl->overflow & OVF_RERUN) return;
  // workgroup b < NB first reduces partition b if it was not split (no queue),
  // then all workgroups take oversized sub-buckets from the work list
  const uint32_t NBIG = (uint32_t)w.ctl->n_big;
  uint32_t max_kk = 0;
#ifdef MOX_RED_STATS  // per-wave cycles: [0] between chunks (loop, load waits) [1] hash [2] fast path [3] slow path
  uint64_t rcyc[4] = {0, 0, 0, 0}, rprev = __builtin_amdgcn_s_memtime();
#define RED_MARK(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); rcyc[k] += t_ - rprev; rprev = t_; } while (0)
#else
#define RED_MARK(k) do { } while (0)
#endif
  const uint32_t ob = blockIdx.x < NB ? w.red_order[blockIdx.x] : 0u;  // k_unit_scan: biggest partitions first
  bool own = blockIdx.x < NB && w.b_kk[ob] == 0;
  for (;;) {
    uint32_t u;
    if (own) {
      u = w.u_base[ob];
      own = false;
    } else {
      if (tid == 0) {
        const uint32_t t = (uint32_t)atomicAdd(&w.ctl->red_ticket, 1ull);
        s_unit = t < NBIG ? w.big_units[t] : 0xFFFFFFFFu;
      }
      __syncthreads();
      u = s_unit;
      __syncthreads();
    }
    if (u == 0xFFFFFFFFu) break;
    const UnitDesc ud = w.udesc[u];
    const uint32_t b = ud.part;
    const bool split = ud.in_n != UNIT_WHOLE;
    const uint32_t shift0 = NB_LOG2 + ud.kk;
    uint64_t ws0, ws1;
    const WRec* wsrc;
    if (split) { wsrc = w.split_w; ws0 = ud.win_off; ws1 = ws0 + ud.win_n; }
    else { wsrc = w.w_sorted; ws0 = w.w_off[b]; ws1 = w.w_off[b + 1]; }
    const uint64_t out0 = ud.rec_off;
    // split unit: its contiguous cold range is cut into NWV wave chunks
    const uint64_t kin0 = split ? ud.in_off : 0;
    const uint32_t kin_n = split ? ud.in_n : 0;
    const bool stamp = MOX_ABL(w.dbg, DBG_STAMP) && tid == 0 && !split;
    if (stamp) w.stamps[b * 8 + 0] = __builtin_amdgcn_s_memrealtime();
    uint32_t kk = 0;
    uint64_t written = 0, wbytes = 0;
    bool failed = false;
    for (uint32_t sub = 0; sub < (1u << kk);) {
      for (int i = tid; i < RED_SLOTS; i += RED_THREADS) {
        tags[i] = 0;
        s.cnt[i] = 0;
      }
      if (tid == 0) { s.misc[0] = 0; s.misc[1] = 0; s.misc[2] = 0; s.misc[3] = 0; }
      // region prefix of a whole partition (the map workgroups' regions one after
      // another), in the sort index / bin space, which is free until the sort
      bool tab = false;  // ticket -> region table built (MOX_RED_TAB)
      if (!split) {
        uint64_t tot;
        const uint32_t cn = tid < (int)G ? cold_n_at(w, G, tid, b) : 0u;
        const uint64_t ex = block_exscan(cn, red_wsum, tot);
        if (tid < (int)G) rpre[tid] = (uint32_t)ex;
        if (tid == 0) rpre[G] = (uint32_t)tot;
#if MOX_RED_DYN && MOX_RED_TAB
        // region of every ticket start (record j RED_TICKET): the region holding
        // it, written by that region's thread from its own prefix and count, so
        // a wave finds a ticket's region in one LDS read instead of a binary
        // search over the prefix (8 dependent reads at 256 regions)
        tab = (tot + RED_TICKET - 1) / RED_TICKET <= (uint64_t)RED_TAB_MAX;
        if (tab && cn) {
          for (uint32_t j = (uint32_t)((ex + RED_TICKET - 1) / RED_TICKET); (uint64_t)j * RED_TICKET < ex + cn; j++)
            rtab[j] = (uint16_t)tid;
        }
#endif
      }
      __syncthreads();
      for (int rep = 0; rep < (MOX_ABL(w.dbg, DBG_RED_TWICE) ? 2 : 1); rep++)
      // cold records: the unit's records as one flat index space (whole
      // partition: region g = map workgroup g, at rpre[g]; split unit: one
      // contiguous range), cut into NWV equal wave shares in 64-record steps so
      // the waves finish together and every chunk is full but the wave's last.
      // Each lane walks forward through the regions (its records ascend by 64
      // per step), the next chunk's loads in flight while the current one is
      // inserted.
      {
#if MOX_RED_DYN
        if (rep) {  // DBG_RED_TWICE: the chunk tickets restart for the second stream
          __syncthreads();
          if (tid == 0) s.misc[2] = 0;
          __syncthreads();
        }
#endif
        const uint32_t n = split ? kin_n : rpre[G];
        constexpr uint32_t CH = 64 * RED_UNROLL;
        // in_sub as one masked compare: hash bits [32 - shift0 - kk, 32 - shift0)
        // equal sub (shift0 + kk <= 32 in every pass that runs; kk == 0: all)
        const uint32_t sub_mask = kk ? ((1u << kk) - 1u) << (32 - shift0 - kk) : 0u;
        const uint32_t sub_val = kk ? sub << (32 - shift0 - kk) : 0u;
#if MOX_RED_DYN
        // dynamic shares: waves take the next 2 chunks from an LDS ticket, so
        // they finish within ~2 chunks of each other (static equal shares left
        // the slowest wave ~25 us behind per partition at C2,
        // profiles/r03_k_reduce_stamps.txt: insert_tail)
        constexpr uint32_t SCH = RED_TICKET;
        static_assert(RED_TICKET == MOX_RED_DEPTH * CH, "a ticket is MOX_RED_DEPTH chunks");
        const uint32_t a1 = n;
        auto grab = [&]() -> uint32_t {
          uint32_t v = 0;
          if (lane == 0) v = lds_fetch_add_lane(&s.misc[2], SCH);
          return __builtin_amdgcn_readfirstlane(v);
        };
        const uint32_t a0 = grab();
#else
        const uint32_t per = (((n + NWV - 1) / NWV) + 63) & ~63u;
        const uint32_t a0 = (uint32_t)wv * per < n ? (uint32_t)wv * per : n;
        const uint32_t a1 = n - a0 < per ? n : a0 + per;
#endif
        const uint4* ubase = split ? w.split_k + kin0 : w.cold + b * RC;  // region g at + g NB RC
        const uint64_t gstride = (uint64_t)NB * RC;
        // lane state: region r holds flat records [rs, re).  (A per-lane 64-bit
        // region base instead of the multiply-add per load cost 2 VGPRs, which
        // at 64 VGPRs doubled the scratch spills.)
        uint32_t r = 0, rs = 0, re = split ? 0xFFFFFFFFu : 0u;
        auto seek = [&](uint32_t c) {  // region of record c: last r with rpre[r] <= c (wave-uniform search)
          if (split || c >= a1) return;
          if (tab) {  // c is a ticket start
            r = rtab[c / SCH];
          } else {
            uint32_t lo = 0, hi = G - 1;
            while (lo < hi) {
              const uint32_t mid = (lo + hi + 1) >> 1;
              if (rpre[mid] <= c) lo = mid; else hi = mid - 1;
            }
            r = lo;
          }
          rs = rpre[r];
          re = rpre[r + 1];
        };
        seek(a0);
        // the walk state is settled before the first record load: a value of it
        // still arriving from a register reload (scratch is vector memory) made
        // the compiler wait for every load in flight at each chunk (vmcnt(0))
        asm volatile("" ::"v"(r), "v"(rs), "v"(re));
        typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
        auto load = [&](uint32_t c, uint4 (&v)[RED_UNROLL]) {  // unconditional: uniform vmcnt
          // every address first, then the loads back to back: a region walk
          // between two loads of one chunk made the compiler wait for the first
          // (its temporaries reused the in-flight load's registers)
          const uint4* p[RED_UNROLL];
#pragma unroll
          for (int u2 = 0; u2 < RED_UNROLL; u2++) {
            const uint32_t i = c + u2 * 64 + lane;
            const bool ok = i < a1;
            bool adv = ok && i >= re;
            // per-lane walk to the region holding record i: one step covers a
            // chunk that crosses one region end (regions average ~150 records);
            // the loop only runs for regions of fewer than 64 records (the
            // compiler put a wait for every load in flight at the head of a
            // loop here, so the common step stays outside it)
            if (adv) { r++; rs = re; re = rpre[r + 1]; }
            adv = ok && i >= re;
            if (__any(adv)) {
              do {
                if (adv) { r++; rs = re; re = rpre[r + 1]; }
                adv = ok && i >= re;
              } while (__any(adv));
            }
            p[u2] = ok ? ubase + (uint64_t)r * gstride + (i - rs) : ubase;
          }
#pragma unroll
          for (int u2 = 0; u2 < RED_UNROLL; u2++) {
            const u32x4 x = *reinterpret_cast<const u32x4*>(p[u2]);
            v[u2] = make_uint4(x.x, x.y, x.z, x.w);
          }
        };
        auto process = [&](const uint4 (&cur)[RED_UNROLL], uint32_t c) {
          if (__hip_atomic_load(&s.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP)) {  // redone anyway
            // the chunk's loads are waited for on this path too: left pending
            // into the next iteration, they made the compiler wait for every
            // load in flight (vmcnt(0)) before the region walk, each chunk
#pragma unroll
            for (int u2 = 0; u2 < RED_UNROLL; u2++) asm volatile("" ::"v"(cur[u2].x), "v"(cur[u2].y), "v"(cur[u2].z), "v"(cur[u2].w));
            return;
          }
          uint32_t h[RED_UNROLL];
          bool todo[RED_UNROLL];
          RED_MARK(0);
#pragma unroll
          for (int u2 = 0; u2 < RED_UNROLL; u2++) {
            h[u2] = hash32(cur[u2].x, cur[u2].y, cur[u2].z, cur[u2].w);
            todo[u2] = c + u2 * 64 + lane < a1 && ((h[u2] ^ sub_val) & sub_mask) == 0u;  // in_sub
          }
          RED_MARK(1);
          if (!MOX_ABL(w.dbg, DBG_RED_NOINSERT)) {
            uint32_t nnew = 0;
#pragma unroll
            for (int u2 = 0; u2 < RED_UNROLL; u2++) {
              int r = RED_MISS;
              if (todo[u2]) r = red_try(s, h[u2], cur[u2], 1);
              todo[u2] = todo[u2] && r == RED_MISS;
              nnew += (uint32_t)__popcll(__ballot(r == RED_NEW));
            }
            // the chunk's new keys counted at once (one lane, one LDS atomic);
            // past RED_CAP the unit is redone in sub-passes
            if (nnew && lane == 0) {
#if MOX_RED_LAZYCAP
              lds_add_lane(&s.misc[0], nnew);  // the RED_CAP test once the stream is done
#else
              const uint32_t u0 = lds_fetch_add_lane(&s.misc[0], nnew);
              if (u0 + nnew > (uint32_t)RED_CAP) s.misc[1] = 1;
#endif
            }
            RED_MARK(2);
#pragma unroll
            for (int u2 = 0; u2 < RED_UNROLL; u2++)
              if (todo[u2] && !MOX_ABL(w.dbg, DBG_RED_NOSLOW)) {
                if (s.dbg) atomicAdd(&s.dbg[3], 1u);  // cold-stream lanes on the slow path
                red_insert(s, h[u2], cur[u2], 1);
              }
            RED_MARK(3);
          } else {
#pragma unroll
            for (int u2 = 0; u2 < RED_UNROLL; u2++) asm volatile("" ::"v"(h[u2]));
          }
        };
        uint32_t c = a0;
        uint4 A[RED_UNROLL], B[RED_UNROLL];
#if MOX_RED_DYN && MOX_RED_DEPTH == 3
        // tickets of three chunks [c, c + CH), [c + CH, c + 2 CH), [c + 2 CH,
        // c + 3 CH): two chunks' loads in flight while one is inserted (the
        // stream is bound by the bytes each wave keeps in flight)
        uint4 C[RED_UNROLL];
        if (c < a1) {
          load(c, A);
          load(c + CH, B);
        }
        while (c < a1) {
          load(c + 2 * CH, C);
          uint32_t tv = 0;
          if (lane == 0) tv = lds_fetch_add_lane(&s.misc[2], SCH);
          process(A, c);
          const uint32_t cn = __builtin_amdgcn_readfirstlane(tv);
          seek(cn);
          load(cn, A);
          process(B, c + CH);
          load(cn + CH, B);
          process(C, c + 2 * CH);
          c = cn;
        }
#elif MOX_RED_DYN
        // chunk pairs [c, c + CH), [c + CH, c + SCH) of one ticket, the next
        // ticket's first chunk in flight while the second is inserted
        if (c < a1) load(c, A);
        while (c < a1) {
          load(c + CH, B);
          // the next ticket's LDS atomic goes out before this chunk's probes
          uint32_t tv = 0;
          if (lane == 0) tv = lds_fetch_add_lane(&s.misc[2], SCH);
          process(A, c);
          const uint32_t cn = __builtin_amdgcn_readfirstlane(tv);
          seek(cn);
          load(cn, A);
          process(B, c + CH);
          c = cn;
        }
#else
        if (c < a1) load(c, A);
        while (c < a1) {
          load(c + CH, B);
          process(A, c);
          c += CH;
          if (c >= a1) break;
          load(c + CH, A);
          process(B, c);
          c += CH;
        }
#endif
      }
      if (stamp) w.stamps[b * 8 + 1] = __builtin_amdgcn_s_memrealtime();  // wave 0 done streaming
      for (uint64_t i = ws0 + tid; i < ws1; i += RED_THREADS) {
        const WRec rr = wsrc[i];
        const uint4 k = make_uint4((uint32_t)rr.w0, (uint32_t)(rr.w0 >> 32), (uint32_t)rr.w1, (uint32_t)(rr.w1 >> 32));
        const uint32_t h = hash32(k.x, k.y, k.z, k.w);
        if (!__hip_atomic_load(&s.misc[1], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP) && in_sub(h, shift0, kk, sub)) {
          const int r = red_try(s, h, k, rr.count);
          if (r == RED_MISS) {
            red_insert(s, h, k, rr.count);
          } else if (r == RED_NEW) {
            const uint32_t u0 = atomicAdd(&s.misc[0], 1u);
            if (u0 >= (uint32_t)RED_CAP) s.misc[1] = 1;
          }
        }
      }
      // The chunks' new-key counts went out as inline-asm LDS adds, which the
      // compiler's wait-count tracking does not see: drain the DS queue
      // explicitly, so the barrier's release cannot be dropped as "nothing
      // pending" and misc[0] is settled when it is read below.
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __syncthreads();
#ifdef MOX_CHECK
      {  // table invariants red_try relies on: every bucket's taken slots are a
         // prefix, and no key sits in two slots of its two buckets
        bool ok = true;
        for (int bk = tid; bk < RED_BUCKETS; bk += RED_THREADS) {
          for (int i = 0; i < 4; i++) {
            const uint32_t t = tags[4 * bk + i];
            if (t == 0) {
              for (int j = i + 1; j < 4; j++) ok = ok && tags[4 * bk + j] == 0;
              continue;
            }
            const int lim = bk + 1 < RED_BUCKETS ? 8 : 4;
            for (int j = i + 1; j < lim; j++)
              if (tags[4 * bk + j] == t && key_eq16(s.key[4 * bk + j], s.key[4 * bk + i])) ok = false;
          }
        }
        (void)MOX_CHK(w, ok, CHK_RED_TABLE);
      }
#endif
#if MOX_RED_LAZYCAP
      if (s.misc[0] > (uint32_t)RED_CAP) {  // (uniform: every thread reads the settled count)
        __syncthreads();
        if (tid == 0) s.misc[1] = 1;
        __syncthreads();
      }
#endif
      if (s.misc[1]) {  // too many distinct keys for one table: split further, redo the unit
        kk++;
        // the redo does not see this attempt's keys (readers take a slot's key
        // only after its published count, and counts restart at 0; cleared
        // anyway, so no stale key ever sits in a slot being claimed)
        for (int i = tid; i < RED_SLOTS; i += RED_THREADS) s.key[i] = make_uint4(0, 0, 0, 0);
        __syncthreads();
        if (shift0 + kk > 32) {  // > RED_CAP distinct keys share every hash bit: cannot split
          if (tid == 0) atomicOr(&w.ctl->overflow, OVF_REDUCE);
          failed = true;
          break;
        }
        sub = 0;
        written = 0;
        wbytes = 0;
        continue;
      }
      // deterministic order (key_less): bucket sort by the hash bits below the
      // unit and sub-pass bits, then a key_less insertion sort inside each bin
      if (stamp) w.stamps[b * 8 + 2] = __builtin_amdgcn_s_memrealtime();  // all waves done inserting
      const uint32_t bsh = shift0 + kk;
      for (int i = tid; i < RED_SORTB; i += RED_THREADS) { s.bin[i] = 0; s.fill[i] = 0; }
      __syncthreads();
      for (int i = tid; i < RED_SLOTS; i += RED_THREADS)
        if (tags[i]) {
          const uint32_t bn = red_bin(tags[i], bsh);
          atomicAdd(reinterpret_cast<uint32_t*>(s.bin) + (bn >> 1), 1u << (16 * (bn & 1)));
        }
      __syncthreads();
      {  // exclusive scan of the RED_SORTB bin counts (2 per thread)
        uint64_t tot;
        const uint32_t c0 = s.bin[2 * tid], c1 = s.bin[2 * tid + 1];
        const uint64_t ex = block_exscan(c0 + c1, red_wsum, tot);
        s.bin[2 * tid] = (uint16_t)ex;
        s.bin[2 * tid + 1] = (uint16_t)(ex + c0);
        if (tid == 0) s.bin[RED_SORTB] = (uint16_t)tot;
      }
      __syncthreads();
      // distinct keys = taken slots (the tag count of the bin scan above), not
      // misc[0]: no wave may disagree on it (check builds: the two agree)
      const uint32_t nu = s.bin[RED_SORTB];
      (void)MOX_CHK(w, nu == s.misc[0], CHK_RED_NU);
      for (int i = tid; i < RED_SLOTS; i += RED_THREADS)
        if (tags[i]) {
          const uint32_t bn = red_bin(tags[i], bsh);
          const uint32_t old = atomicAdd(reinterpret_cast<uint32_t*>(s.fill) + (bn >> 1), 1u << (16 * (bn & 1)));
          const uint32_t p = s.bin[bn] + ((old >> (16 * (bn & 1))) & 0xFFFFu);
          s.idx[p] = (uint16_t)i;
        }
      __syncthreads();
      if (!MOX_ABL(w.dbg, DBG_RED_NOSORT)) {
        for (int bn = tid; bn < RED_SORTB; bn += RED_THREADS) {
          const uint32_t lo = s.bin[bn], hi = s.bin[bn + 1];
          for (uint32_t i = lo + 1; i < hi; i++) {  // insertion sort of a tiny bin
            const uint16_t x = s.idx[i];
            uint32_t j = i;
            while (j > lo && red_less(s, x, s.idx[j - 1])) { s.idx[j] = s.idx[j - 1]; j--; }
            s.idx[j] = x;
          }
        }
      }
      __syncthreads();
      if (stamp) w.stamps[b * 8 + 3] = __builtin_amdgcn_s_memrealtime();  // sorted
      uint32_t lb = 0;
      for (uint32_t i = tid; i < nu; i += RED_THREADS) {
        const uint16_t sl = s.idx[i];
        const uint4 kk4 = s.key[sl];
        // check builds: the unit's distinct keys stay inside its record range
        if (MOX_CHK(w, written + i < (split ? (uint64_t)ud.in_n + ud.win_n : w.rec_off[b + 1] - w.rec_off[b]) &&
                           out0 + written + i < w.uniq_cap, CHK_RED_OUT)) {
          w.uk[out0 + written + i] = kk4;
          w.uc[out0 + written + i] = s.cnt[sl];
        }
        lb += key_len16(kk4);
      }
      if (lb) atomicAdd(&s.misc[3], lb);
      written += nu;
      sub++;
      lds_barrier();  // the table is re-zeroed next: LDS only, the uk / uc stores need not land first
      if (tid == 0) wbytes += s.misc[3];  // read (and reset at the next sub-pass) by tid 0 only
    }
    if (stamp) {
      w.stamps[b * 8 + 4] = __builtin_amdgcn_s_memrealtime();
      uint32_t hw;
      asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(hw));
      w.stamps[b * 8 + 5] = hw;
      w.stamps[b * 8 + 6] = s.misc[0];
    }
    if (tid == 0) {
      w.u_uniq[u] = failed ? 0 : written;
      w.u_bytes[u] = failed ? 0 : wbytes;
      if (!split) w.b_uniq[b] = failed ? 0 : written;  // split partitions: summed by k_unit_uniq_scan
    }
    if (kk > max_kk) max_kk = kk;
    __syncthreads();
  }
#ifdef MOX_RED_STATS
  if (lane == 0 && w.stamps) {
    unsigned long long* o = w.stamps + 8 * 4096 + 8 * 1024 * MAP_WAVES + ((uint64_t)blockIdx.x * NWV + wv) * 4;
    for (int k = 0; k < 4; k++) o[k] = rcyc[k];
  }
#endif
  if (tid == 0) {
    if (max_kk) atomicMax(&w.ctl->max_sub, 1u << max_kk);
    if (s.dbg) for (int i = 0; i < 8; i++) atomicAdd(&w.ctl->dbg_cnt[i], (unsigned long long)dbgc[i]);
  }
}

// ------------------------------------------------------------------ small-unit reduce
// Geometry of k_reduce_small (small units with weighted records, below).
constexpr int SR_THREADS = 128;
constexpr int SR_PER = SMALL_CAP / SR_THREADS;  // records (and sorted positions) per thread
constexpr int SR_BIN_BITS = 9;
constexpr int SR_BINS = 1 << SR_BIN_BITS;  // hash bits right below the unit bits
static_assert(SR_PER * SR_THREADS == (int)SMALL_CAP && SR_BINS == 4 * SR_THREADS, "k_reduce_small geometry");


struct SmallIn {  // prefetched keys (weighted counts are read at use: rare outside exchange passes)
  uint4 k[SR_PER];
};
// k_reduce_sort1 takes the split units of <= SMALL_CAP records that hold only
// cold (count 1) records; k_reduce_small the small units with weighted records.
__device__ __forceinline__ bool sort1_unit(const UnitDesc& d) { return d.in_n != UNIT_WHOLE && d.win_n == 0 && d.in_n <= SMALL_CAP; }
__device__ __forceinline__ bool small_unit(const UnitDesc& d) {
  return d.in_n != UNIT_WHOLE && d.win_n != 0 && d.in_n + d.win_n <= SMALL_CAP;
}
// Descriptor of unit min(u, U - 1): no select on the loaded value, so the load
// stays in flight until first use (the caller checks u < U there).
__device__ __forceinline__ UnitDesc load_desc(const Work& w, uint32_t u, uint32_t U) { return w.udesc[u < U ? u : U - 1]; }
// Branch-free raw key loads (one address select per slot, invalid slots read
// a valid dummy address, no select on loaded values): the compiler leaves them
// in flight until the next iteration uses them.
__device__ __forceinline__ void load_small(const Work& w, const UnitDesc& d, bool ok, SmallIn& in) {
  const uint32_t nk = d.in_n, n = d.in_n + d.win_n;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
#pragma unroll
  for (int j = 0; j < SR_PER; j++) {
    const uint32_t i = threadIdx.x + j * SR_THREADS;
    const bool valid = ok && i < n, cold = i < nk;
    const uint8_t* kp = cold ? reinterpret_cast<const uint8_t*>(w.split_k + d.in_off + i)
                             : reinterpret_cast<const uint8_t*>(w.split_w + d.win_off + (i - nk));
    if (!valid) kp = reinterpret_cast<const uint8_t*>(w.split_k);
    const u32x4 v = *reinterpret_cast<const u32x4*>(kp);
    in.k[j] = make_uint4(v.x, v.y, v.z, v.w);
  }
}

// Sub-buckets of split partitions with <= SMALL_CAP records (the common case of
// high-cardinality input).  Persistent 128-thread workgroups (8 per CU) take
// units grid-strided (no work queue); the next unit's descriptor and records
// are loaded into registers while the current one is processed.  Per unit:
//  A. records into LDS (key, 32-bit hash, count);
//  B. group by exact key in an LDS open-addressing table of record indices
//     (SR_TSLOTS slots, linear probing, CAS claim): the first record of a key
//     claims a slot and becomes its leader; every other record of that key adds
//     its count to the leader's -- so a word repeated ~70 times in one unit
//     (C4 at 16 GiB: every 4-letter word) costs 70 LDS adds, not the O(c^2)
//     rank of a sort over all records;
//  C. leaders into 512 bins by the 9 hash bits below the unit's bits (counting
//     sort), each leader ranked by key_less among the few leaders of its bin;
//  D. distinct keys written in key_less order, as k_reduce.
// Barriers are LDS-only (s_waitcnt lgkmcnt(0); s_barrier), so pending global
// stores are never waited for.
constexpr int SR_TSLOTS = 1024;  // u16 record indices, two per LDS word; > SMALL_CAP: every record can lead
constexpr uint32_t SR_EMPTY16 = 0xFFFFu;
static_assert(SR_TSLOTS >= 2 * (int)SMALL_CAP && SR_TSLOTS == 8 * SR_THREADS, "k_reduce_small table");
__device__ __forceinline__ uint32_t sr_slot(uint32_t h) { return (h * 0x9E3779B1u) >> (32 - 10); }  // SR_TSLOTS = 2^10

extern "C" __global__ __launch_bounds__(SR_THREADS, 4) void k_reduce_small(Work w) {  // 8 per CU (4 waves/SIMD): <= 128 VGPRs
  __shared__ uint4 key[SMALL_CAP];
  __shared__ unsigned long long acc[SMALL_CAP];  // record count; a leader's: its key's total
  __shared__ uint32_t hh[SMALL_CAP];
  __shared__ uint32_t tab[SR_TSLOTS / 2];         // leader record index per slot, u16 pairs (0xFFFF = free)
  __shared__ uint16_t idx2[SMALL_CAP];            // leaders in key_less order
  __shared__ uint32_t bins[SR_BINS / 2];          // u16 pairs: leader counts, then exclusive starts
  __shared__ uint32_t wsa[SR_THREADS / 64];
  __shared__ uint32_t sbytes;
  uint16_t* idx = reinterpret_cast<uint16_t*>(tab);  // leaders grouped by bin (the table is dead by then)
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  if (w.ctl->overflow & OVF_RERUN) return;
  const uint32_t U = (uint32_t)w.ctl->n_units;
  const uint32_t NS = (uint32_t)w.ctl->n_small;  // work list (k_split_scatter): the small units with weighted records
  auto uid = [&](uint32_t t) { return w.small_units[t < NS ? t : NS - 1]; };
  const uint32_t G = gridDim.x;
  uint16_t* bin16 = reinterpret_cast<uint16_t*>(bins);
  __shared__ UnitDesc dring[2];  // descriptors of this and the next unit (written one unit ahead)
  uint32_t t = blockIdx.x;
  if (t >= NS) return;
  if (tid == 0) { dring[0] = load_desc(w, uid(t), U); dring[1] = load_desc(w, uid(t + G), U); sbytes = 0; }
  bins[tid] = 0;
  bins[tid + SR_THREADS] = 0;
#pragma unroll
  for (int q = 0; q < SR_TSLOTS / 2 / SR_THREADS; q++) tab[tid + q * SR_THREADS] = 0xFFFFFFFFu;
  lds_barrier();
  SmallIn in;
  {
    const UnitDesc d0 = dring[0];
    load_small(w, d0, small_unit(d0), in);
  }
#ifdef MOX_SR_STATS
  uint64_t cyc[4] = {0, 0, 0, 0}, tprev = __builtin_amdgcn_s_memtime();
#define SR_MARK(k) do { const uint64_t t_ = __builtin_amdgcn_s_memtime(); cyc[k] += t_ - tprev; tprev = t_; } while (0)
#else
#define SR_MARK(k) do { } while (0)
#endif
  for (uint32_t it = 0; t < NS; t += G, it++) {
    const uint32_t u = uid(t);
    const UnitDesc d = dring[it & 1], dn = dring[(it + 1) & 1];
    bool cur_small = small_unit(d);
    // check builds: the unit's input and output ranges lie inside their buffers
    if (cur_small && !MOX_CHK(w, d.in_off + d.in_n <= w.split_k_cap && d.win_off + d.win_n <= w.split_w_cap &&
                                     d.rec_off + d.in_n + d.win_n <= w.uniq_cap, CHK_SMALL_DESC))
      cur_small = false;
    const uint32_t n = d.in_n + d.win_n, nk = d.in_n, shift = NB_LOG2 + d.kk;
    uint32_t h[SR_PER];
    // A. this unit's records into LDS
    if (cur_small) {
#pragma unroll
      for (int j = 0; j < SR_PER; j++) {
        const uint32_t i = tid + j * SR_THREADS;
        h[j] = hash32(in.k[j].x, in.k[j].y, in.k[j].z, in.k[j].w);
        if (i < n) {
          key[i] = in.k[j];
          hh[i] = h[j];
          acc[i] = i < nk ? 1ull : w.split_w[d.win_off + (i - nk)].count;
        }
      }
    }
    // the next unit's records and the descriptor after it: in flight during this unit
    SmallIn inn;
    load_small(w, dn, t + G < NS && small_unit(dn), inn);
    UnitDesc dnn;
    if (tid == 0) dnn = load_desc(w, uid(t + 2 * G), U);
    if (cur_small) {
      lds_barrier();
      SR_MARK(0);
      // B. group by key: claim a slot, or add to the leader holding this key.
      // The thread's records are probed in one interleaved loop (one probe step
      // per iteration, moving to its next record when one is placed), so a
      // wave iterates max over lanes of the sum of its probe lengths rather
      // than the sum over records of the wave's longest probe.
      {
        uint32_t j = 0, sl = sr_slot(h[0]);
        uint32_t i = tid;
        bool more = i < n;
        while (__builtin_amdgcn_ballot_w64(more) != 0) {
          if (more) {
            uint4 k = in.k[0];
            uint32_t hj = h[0];
#pragma unroll
            for (int q = 1; q < SR_PER; q++)
              if (j == (uint32_t)q) { k = in.k[q]; hj = h[q]; }
            const uint32_t wi = sl >> 1, sh = 16 * (sl & 1);
            uint32_t v = __hip_atomic_load(&tab[wi], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WORKGROUP);
            uint32_t cur = (v >> sh) & 0xFFFFu;
            bool placed = false;
            if (cur == SR_EMPTY16) {
              const uint32_t old = atomicCAS(&tab[wi], v, (v & ~(0xFFFFu << sh)) | (i << sh));
              if (old == v) placed = true;   // this record leads its key
              else cur = (old >> sh) & 0xFFFFu;  // lost the race (or the other half changed): look again
            }
            if (!placed && cur != SR_EMPTY16) {
              if (hh[cur] == hj && key_eq16(key[cur], k)) {
                atomicAdd(&acc[cur], acc[i]);
                placed = true;
              } else {
                if (hh[cur] == hj) MOX_PATH(w.ctl, PATH_SMALL_TAG);  // same hash, another key
                sl = (sl + 1) & (SR_TSLOTS - 1);
              }
            }
            if (placed) {
              j++;
              i += SR_THREADS;
              more = j < (uint32_t)SR_PER && i < n;
              uint32_t hn = h[0];
#pragma unroll
              for (int q = 1; q < SR_PER; q++)
                if (j == (uint32_t)q) hn = h[q];
              sl = sr_slot(hn);
            }
          }
        }
      }
      lds_barrier();
      SR_MARK(1);
      // C. leaders (table slots) into bins; arrival rank inside the bin.
      // Thread t reads table words t, t + 128, t + 256, t + 384 (8 slots).
      constexpr int SQ = SR_TSLOTS / SR_THREADS;  // slots per thread
      uint32_t L[SQ], rkk[SQ], bnn[SQ];
#pragma unroll
      for (int q = 0; q < SQ / 2; q++) {
        const uint32_t v = tab[tid + q * SR_THREADS];
        L[2 * q] = v & 0xFFFFu;
        L[2 * q + 1] = v >> 16;
      }
#pragma unroll
      for (int q = 0; q < SQ; q++) {
        rkk[q] = 0;
        bnn[q] = 0;
        if (L[q] != SR_EMPTY16) {
          bnn[q] = hbits(hh[L[q]], shift, SR_BIN_BITS);
          const uint32_t old = atomicAdd(&bins[bnn[q] >> 1], 1u << (16 * (bnn[q] & 1)));
          rkk[q] = (old >> (16 * (bnn[q] & 1))) & 0xFFFFu;
        }
      }
      lds_barrier();
      uint32_t nu;
      {  // exclusive scan of the bin counts: bins 4t..4t+3 per thread
        const uint32_t p0 = bins[2 * tid], p1 = bins[2 * tid + 1];
        const uint32_t c0 = p0 & 0xFFFFu, c1 = p0 >> 16, c2 = p1 & 0xFFFFu, c3 = p1 >> 16;
        const uint32_t incl = wave_incl_scan(c0 + c1 + c2 + c3);
        if (lane == 63) wsa[wv] = incl;
        lds_barrier();
        uint32_t ex = incl - (c0 + c1 + c2 + c3);
        nu = 0;
        for (int k = 0; k < SR_THREADS / 64; k++) { if (k < wv) ex += wsa[k]; nu += wsa[k]; }
        bins[2 * tid] = ex | ((ex + c0) << 16);
        bins[2 * tid + 1] = (ex + c0 + c1) | ((ex + c0 + c1 + c2) << 16);
      }
      lds_barrier();
      // leaders grouped by bin (idx overlays the table, read completely above)
#pragma unroll
      for (int q = 0; q < SQ; q++)
        if (L[q] != SR_EMPTY16) idx[bin16[bnn[q]] + rkk[q]] = (uint16_t)L[q];
      lds_barrier();
      // final position: bin start + rank by (h32, hash32b, key) among the bin's leaders
      // (distinct keys: the order is strict; bins hold ~0.6 leaders on average)
#pragma unroll
      for (int q = 0; q < SQ; q++) {
        if (L[q] == SR_EMPTY16) continue;
        const uint32_t x = L[q];
        const uint32_t lo = bin16[bnn[q]], hi = bnn[q] + 1 < SR_BINS ? bin16[bnn[q] + 1] : nu;
        uint32_t r = 0;
        if (hi - lo > 1) {
          const uint32_t hx = hh[x];
          const uint4 kx = key[x];
          for (uint32_t m = lo; m < hi; m++) {
            const uint32_t y = idx[m];
            r += key_less(hh[y], key[y], hx, kx) ? 1u : 0u;
          }
        }
        idx2[lo + r] = (uint16_t)x;
      }
      lds_barrier();
      SR_MARK(2);
      // D. distinct keys out; reset the table and the bins for the next unit
      uint32_t lb = 0;
#pragma unroll
      for (int q = 0; q < SR_PER; q++) {
        const uint32_t p = tid + q * SR_THREADS;
        if (p < nu) {
          const uint32_t x = idx2[p];
          const uint4 k = key[x];
          if (MOX_CHK(w, p < n && d.rec_off + p < w.uniq_cap, CHK_SMALL_OUT)) {  // distinct keys <= records
            w.uk[d.rec_off + p] = k;
            w.uc[d.rec_off + p] = acc[x];
          }
          lb += key_len16(k);
        }
      }
      if (lb) atomicAdd(&sbytes, lb);
      if (tid == 0) w.u_uniq[u] = nu;  // summed per partition by k_unit_uniq_scan
      lds_barrier();  // every read of idx (= the table) is done before the table is reset
      bins[tid] = 0;
      bins[tid + SR_THREADS] = 0;
#pragma unroll
      for (int q = 0; q < SR_TSLOTS / 2 / SR_THREADS; q++) tab[tid + q * SR_THREADS] = 0xFFFFFFFFu;
    } else {
      // A unit this kernel skips (whole partition or > SMALL_CAP records) has
      // no barrier above: without this one, wave 0 could overwrite
      // dring[it & 1] before a lagging wave has read it as d at the top of
      // this iteration.  That wave would then take unit u + 2G for u, disagree
      // with the others on cur_small, pair its barriers with theirs and write
      // its results to wrong (possibly out-of-range) uk / uc positions: the
      // intermittent illegal-address faults of round 1.
      lds_barrier();
    }
    if (tid == 0) dring[it & 1] = dnn;
    lds_barrier();  // LDS reused by the next unit
    if (cur_small && tid == 0) { w.u_bytes[u] = sbytes; sbytes = 0; }  // next adds come after >= 5 barriers
    SR_MARK(3);
    in = inn;
  }
#ifdef MOX_SR_STATS
  if ((tid & 63) == 0)
    for (int k = 0; k < 4; k++) atomicAdd(&w.ctl->dbg_cnt[k], (unsigned long long)cyc[k]);
#endif
#undef SR_MARK
}

// ------------------------------------------------------------------ single-wave sort reduce
// k_reduce_sort1: every split unit of <= SMALL_CAP count-1 records (the bulk of
// high-cardinality input: C4 at 16 GiB has 4.2 M units of ~370 records) is
// reduced by ONE wave, with no workgroup barrier at all:
//  1. its records are loaded (8 per lane, coalesced) into the wave's LDS key
//     array, and each becomes a 32-bit sort key: 23 bits of (the key hash's
//     bits below the unit bits, hash32b), then the record index (9 bits;
//     padding = ~0 sorts last);
//  2. a bitonic sort of the 512 keys in registers (8 per lane; in-lane
//     compare-exchanges, cross-lane ones by DPP or ds_bpermute);
//  3. runs of equal hash bits are the keys' repeats: run heads (verified by
//     comparing the 16-byte keys of every adjacent pair) are compacted by a
//     wave prefix sum, run lengths come from the next head's position, and the
//     distinct keys are written in sort order.
// A unit where two different keys share the 23 sort-key hash bits (about 0.5 %
// of C4's units) is sorted again on 64-bit keys (all of both hashes); only a
// full (h32, hash32b) collision goes on k_reduce's work list (big_units),
// which resolves it exactly.  The sort-key order is the table order every
// reduce kernel uses (key_less).
constexpr int S1_PER = SMALL_CAP / 64;  // records per lane
constexpr int S1_WAVES = 4;             // waves per workgroup, one unit each
static_assert(S1_PER == 8, "k_reduce_sort1: 8 records per lane");
constexpr int S2_PER = 2 * S1_PER;      // k_reduce_sort2: units of SMALL_CAP + 1 .. 2 SMALL_CAP records
// value of lane (lane ^ M)
template <int M>
__device__ __forceinline__ uint32_t xor_lane(uint32_t v) {
  if constexpr (M == 1) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0xB1, 0xF, 0xF, false);   // quad_perm [1,0,3,2]
  if constexpr (M == 2) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x4E, 0xF, 0xF, false);   // quad_perm [2,3,0,1]
  if constexpr (M == 8) return (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x128, 0xF, 0xF, false);  // row_ror:8
  return (uint32_t)__shfl_xor((int)v, M);
}
template <int M>
__device__ __forceinline__ uint64_t xor_lane(uint64_t v) {
  return ((uint64_t)xor_lane<M>((uint32_t)(v >> 32)) << 32) | xor_lane<M>((uint32_t)v);
}
// Bitonic sort of 64 x PER values in registers, position p = lane * PER + s.
// Compare-exchange with the lane (lane ^ M): the lower lane keeps the minimum
// when this block sorts ascending.  k_reduce_sort2's 32-bit keys (16 per
// lane) use min / max with the DPP fused in and one per-stage lane mask: no
// compare + mask XOR per element, whose SALU write of VCC and DPP source move
// cost wait states between VALU instructions (k_reduce_sort2 772 -> 670 us at
// C4).  k_reduce_sort1 keeps compare + select: the same change made it 2-4 %
// slower (it is not issue-bound).
template <int M, int PER, class T>
__device__ __forceinline__ void s1_cross(T (&v)[PER], int lane, uint32_t k) {
  const bool keep_min = ((lane & M) == 0) == (((uint32_t)(lane * PER) & k) == 0);
  if constexpr (sizeof(T) == 4 && PER == 16) {
#pragma unroll
    for (int s = 0; s < PER; s++) {
      const uint32_t pv = xor_lane<M>((uint32_t)v[s]);
      const uint32_t lo = min((uint32_t)v[s], pv), hi = max((uint32_t)v[s], pv);
      v[s] = keep_min ? lo : hi;
    }
  } else {
#pragma unroll
    for (int s = 0; s < PER; s++) {
      const T pv = xor_lane<M>(v[s]);
      v[s] = ((pv < v[s]) == keep_min) ? pv : v[s];
    }
  }
}
template <int PER, class T>
__device__ __forceinline__ void s1_inlane(T (&v)[PER], int lane, uint32_t k, int j) {
#pragma unroll
  for (int s = 0; s < PER; s++) {
    const int t = s ^ j;
    if (t > s) {
      const bool asc = ((uint32_t)(lane * PER + s) & k) == 0;
      const T a = v[s], b = v[t];
      if constexpr (sizeof(T) == 4 && PER == 16) {
        const T lo = a < b ? a : b, hi = a < b ? b : a;
        v[s] = asc ? lo : hi;
        v[t] = asc ? hi : lo;
      } else {
        const bool sw = (a > b) == asc;
        v[s] = sw ? b : a;
        v[t] = sw ? a : b;
      }
    }
  }
}
template <int PER, class T>
__device__ __forceinline__ void s1_sort(T (&v)[PER], int lane_in) {
  // the per-stage lane masks are recomputed in every sort (one compare each)
  // instead of being hoisted out of the unit loop, where ~45 live SGPR pairs
  // spill into VGPR lanes
  int lane = lane_in;
  if constexpr (PER == 16) asm volatile("" : "+v"(lane));
#pragma unroll
  for (uint32_t k = 2; k <= 64u * PER; k <<= 1) {
#pragma unroll
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      if (j >= (uint32_t)PER) {
        switch (j / PER) {
          case 1: s1_cross<1, PER, T>(v, lane, k); break;
          case 2: s1_cross<2, PER, T>(v, lane, k); break;
          case 4: s1_cross<4, PER, T>(v, lane, k); break;
          case 8: s1_cross<8, PER, T>(v, lane, k); break;
          case 16: s1_cross<16, PER, T>(v, lane, k); break;
          default: s1_cross<32, PER, T>(v, lane, k); break;
        }
      } else {
        s1_inlane<PER, T>(v, lane, k, (int)j);
      }
    }
  }
}

// One count-1 unit (n <= 64 PER records, keys k[s] = record s * 64 + lane)
// reduced by one wave: key[] / hp[] are the wave's LDS arrays (64 PER keys,
// 64 PER + 2 run heads).  IB index bits; the 32-bit sort key keeps 32 - IB
// bits of (h32 below the unit bits, hash32b).
template <int PER>
__device__ __forceinline__ void sort_reduce_unit(const Work& w, uint32_t u, const UnitDesc& d, const uint4 (&k)[PER],
                                                 uint4* key, uint16_t* hp, int lane) {
  constexpr uint32_t N = 64u * PER, IB = PER == 8 ? 9u : 10u, IM = N - 1;
  static_assert((1u << IB) == N, "index bits");
  const uint32_t n = d.in_n, shift = NB_LOG2 + d.kk;
  uint32_t v[PER];
#pragma unroll
  for (int s = 0; s < PER; s++) {
    const uint32_t i = (uint32_t)(s * 64 + lane);
    const uint32_t h = hash32(k[s].x, k[s].y, k[s].z, k[s].w), hb = hash32b(k[s].x, k[s].y, k[s].z, k[s].w);
    // sort key: the top 32 - IB bits of (h32 bits below the unit, hash32b) --
    // the leading bits of the table order key_less -- then the record index.
    // Padding ~0 cannot tie a real key: with padding present every real index
    // is <= N - 2.
    const uint32_t pre = (h << shift) | (hb >> (32 - shift));
    v[s] = i < n ? ((pre & ~IM) | i) : ~0u;
    if (i < n) key[i] = k[s];
  }
  s1_sort<PER, uint32_t>(v, lane);
  if (MOX_ABL(w.dbg, DBG_S1_SORT2)) s1_sort<PER, uint32_t>(v, lane);
  // run heads: hash bits differ from the previous position's
  uint32_t idx[PER];
  uint32_t hm = 0, bad = 0;
  wave_lds_fence();  // key[] written by every lane
  {
    uint32_t prev = from_prev_lane(v[PER - 1]);
#pragma unroll
    for (int s = 0; s < PER; s++) {
      const uint32_t p = (uint32_t)(lane * PER + s);
      const bool valid = p < n;
      const bool head = valid && (p == 0 || (v[s] >> IB) != (prev >> IB));
      if (head) hm |= 1u << s;
      if (valid && !head) bad |= key_eq16(key[v[s] & IM], key[prev & IM]) ? 0u : 1u;
      idx[s] = v[s] & IM;
      prev = v[s];
    }
  }
  if (__any(bad != 0)) {
    if (lane == 0) MOX_PATH(w.ctl, PATH_SORT_RESORT);
    // two different keys share the sort-key hash bits (~0.5 % of C4's units):
    // sort again on 64-bit keys -- the h32 bits below the unit, all of
    // hash32b, the index -- which is key_less order whenever (h32, hash32b)
    // differ
    // (keys from the wave's LDS copy: the registers k[] are dead after the
    // first pass, which keeps this rare path from setting the kernel's
    // register peak)
    uint64_t v2[PER];
#pragma unroll
    for (int s = 0; s < PER; s++) {
      const uint32_t i = (uint32_t)(s * 64 + lane);
      const uint4 ks = key[i < n ? i : 0u];
      const uint32_t h = hash32(ks.x, ks.y, ks.z, ks.w), hb = hash32b(ks.x, ks.y, ks.z, ks.w);
      const uint64_t pre = ((uint64_t)(shift >= 32 ? 0u : (h << shift) >> shift) << (32 + IB)) | ((uint64_t)hb << IB);
      v2[s] = i < n ? (pre | i) : ~0ull;
    }
    s1_sort<PER, uint64_t>(v2, lane);
    uint64_t prev = ((uint64_t)from_prev_lane((uint32_t)(v2[PER - 1] >> 32)) << 32) | from_prev_lane((uint32_t)v2[PER - 1]);
    hm = 0;
    bad = 0;
#pragma unroll
    for (int s = 0; s < PER; s++) {
      const uint32_t p = (uint32_t)(lane * PER + s);
      const bool valid = p < n;
      const bool head = valid && (p == 0 || (v2[s] >> IB) != (prev >> IB));
      if (head) hm |= 1u << s;
      if (valid && !head) bad |= key_eq16(key[(uint32_t)v2[s] & IM], key[(uint32_t)prev & IM]) ? 0u : 1u;
      idx[s] = (uint32_t)v2[s] & IM;
      prev = v2[s];
    }
  }
  if (__any(bad != 0)) {  // (h32, hash32b) shared by two keys: k_reduce resolves this unit
    if (lane == 0) {
      MOX_PATH(w.ctl, PATH_SORT_TO_RED);
      const unsigned long long q = atomicAdd(&w.ctl->n_big, 1ull);
      if (MOX_CHK(w, q < U_MAX, CHK_UNIT)) w.big_units[q] = u;
    }
  } else {
    const uint32_t nh = (uint32_t)__popc(hm);
    const uint32_t incl = wave_incl_scan(nh);
    const uint32_t nu = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
    uint32_t o = incl - nh;
#pragma unroll
    for (int s = 0; s < PER; s++)
      if ((hm >> s) & 1u) hp[o++] = (uint16_t)(lane * PER + s);
    if (lane == 0) hp[nu] = (uint16_t)n;
    wave_lds_fence();
    o = incl - nh;
    uint32_t lb = 0;
    // distinct keys as (record index, count) in 4 bytes each: k_mat takes the
    // key bytes from the unit's split_k range (no 24-byte uk / uc round trip)
#pragma unroll
    for (int s = 0; s < PER; s++) {
      if ((hm >> s) & 1u) {
        const uint32_t p = (uint32_t)(lane * PER + s);
        if (MOX_CHK(w, o < n && d.rec_off + o < w.uniq_cap, CHK_SMALL_OUT))
          w.ui[d.rec_off + o] = (idx[s] << 16) | (uint32_t)(hp[o + 1] - p);
        lb += key_len16(key[idx[s]]);
        o++;
      }
    }
    uint32_t tb = lb;
    for (int off = 32; off > 0; off >>= 1) tb += __shfl_xor(tb, off);
    if (lane == 0) {
      w.u_uniq[u] = nu | U_IDX;
      w.u_bytes[u] = tb;
    }
  }  // no collision
  wave_lds_fence();  // this unit's LDS reads before the next unit's writes
}

extern "C" __global__ __launch_bounds__(64 * S1_WAVES, MOX_S1_WG) void k_reduce_sort1(Work w) {
  __shared__ uint4 skey[S1_WAVES][SMALL_CAP];
  __shared__ uint16_t shp[S1_WAVES][SMALL_CAP + 2];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint4* key = skey[wv];
  uint16_t* hp = shp[wv];
  if (w.ctl->overflow & OVF_RERUN) return;
  const uint32_t U = (uint32_t)w.ctl->n_units;
  const uint32_t GW = gridDim.x * S1_WAVES;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  // software pipeline: the next unit's descriptor is loaded one unit ahead and
  // its records are in flight (registers) while this unit is sorted
  auto ok_unit = [&](const UnitDesc& dd) {
    return sort1_unit(dd) && MOX_CHK(w, dd.in_off + dd.in_n <= w.split_k_cap && dd.rec_off + dd.in_n <= w.uniq_cap,
                                     CHK_SMALL_DESC);
  };
  auto load_keys = [&](const UnitDesc& dd, bool ok, uint4 (&kk)[S1_PER]) {
    const uint4* src = w.split_k + (ok ? dd.in_off : 0);
    const uint32_t nn = ok ? dd.in_n : 0u;
#pragma unroll
    for (int s = 0; s < S1_PER; s++) {
      const uint32_t i = (uint32_t)(s * 64 + lane);
      const u32x4 x = *reinterpret_cast<const u32x4*>(src + (i < nn ? i : 0u));
      kk[s] = make_uint4(x.x, x.y, x.z, x.w);
    }
  };
  // descriptors carry only the fields this kernel reads (7 of 10 dwords):
  // three of them are live across the sort, and at 128 VGPRs the full ones
  // spilled to scratch, whose reloads (vector memory) waited for every load
  // and store in flight once per unit
  auto slim = [&](uint32_t uu) {
    const UnitDesc& x = w.udesc[uu < U ? uu : U - 1];
    return UnitDesc{x.in_off, 0, x.rec_off, x.in_n, x.win_n, 0, x.kk};
  };
  uint32_t u = blockIdx.x * S1_WAVES + wv;
  if (u >= U) return;
  UnitDesc d = slim(u);
  UnitDesc dn = slim(u + GW);
  uint4 k[S1_PER];
  load_keys(d, ok_unit(d), k);
  for (; u < U; u += GW) {
    const UnitDesc dnn = slim(u + 2 * GW);
    uint4 kn[S1_PER];
    load_keys(dn, u + GW < U && ok_unit(dn), kn);
    if (ok_unit(d)) sort_reduce_unit<S1_PER>(w, u, d, k, key, hp, lane);
    d = dn;
    dn = dnn;
#pragma unroll
    for (int s = 0; s < S1_PER; s++) k[s] = kn[s];
  }
}

// k_reduce_sort2: the count-1 units of SMALL_CAP + 1 .. 2 SMALL_CAP records
// (listed by k_split_scatter in mid_units; C4 16 GiB: ~2.4 % of its units,
// where a few 4-letter words repeated ~70 times each land in one sub-bucket),
// one wave each with 16 records per lane -- the same reduction as
// k_reduce_sort1 instead of a 1024-thread k_reduce workgroup per unit.
extern "C" __global__ __launch_bounds__(64) void k_reduce_sort2(Work w) {
  __shared__ uint4 key[2 * SMALL_CAP];
  __shared__ uint16_t hp[2 * SMALL_CAP + 2];
  const int lane = threadIdx.x;
  if (w.ctl->overflow & OVF_RERUN) return;
  const uint32_t nm = (uint32_t)w.ctl->n_mid;
  typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
  for (uint32_t t = blockIdx.x; t < nm; t += gridDim.x) {
    const uint32_t u = w.mid_units[t];
    const UnitDesc d = w.udesc[u];
    if (!MOX_CHK(w, d.in_n <= 2 * SMALL_CAP && d.in_off + d.in_n <= w.split_k_cap && d.rec_off + d.in_n <= w.uniq_cap,
                 CHK_SMALL_DESC))
      continue;
    uint4 k[S2_PER];
#pragma unroll
    for (int s = 0; s < S2_PER; s++) {
      const uint32_t i = (uint32_t)(s * 64 + lane);
      const u32x4 x = *reinterpret_cast<const u32x4*>(w.split_k + d.in_off + (i < d.in_n ? i : 0u));
      k[s] = make_uint4(x.x, x.y, x.z, x.w);
    }
    sort_reduce_unit<S2_PER>(w, u, d, k, key, hp, lane);
  }
}

// ------------------------------------------------------------------ table directory
// k_unit_uniq_scan (one workgroup per partition): offsets of a split
// partition's units inside the partition (keys and key bytes) and the
// partition's totals; plus, for long-table slice b, its occupied slots and their
// bytes.  No global atomics in the reduce kernels, whose units of one partition
// run side by side.
__device__ __forceinline__ void unit_uniq_scan(const Work& w) {
  __shared__ uint64_t wsum[16];
  __shared__ unsigned long long lsn, lsb;
  const uint32_t b = blockIdx.x;
  const int tid = threadIdx.x;
  if (w.ctl->overflow & OVF_RERUN) return;
  const uint32_t kk = w.b_kk[b], u0 = w.u_base[b];
  if (!kk) {
    if (tid == 0) { w.u_uniq_off[u0] = 0; w.u_bytes_off[u0] = 0; w.b_bytes[b] = w.u_bytes[u0]; }
  } else {
    const uint32_t nsub = 1u << kk;
    uint64_t v[SUB_PER_T], y[SUB_PER_T], sv = 0, sy = 0;
#pragma unroll
    for (int j = 0; j < SUB_PER_T; j++) {
      const uint32_t sb = SUB_PER_T * tid + j;
      v[j] = sb < nsub ? w.u_uniq[u0 + sb] & ~U_IDX : 0;
      y[j] = sb < nsub ? w.u_bytes[u0 + sb] : 0;
      sv += v[j];
      sy += y[j];
    }
    uint64_t tot, btot;
    uint64_t ex = block_exscan(sv, wsum, tot);
    uint64_t ey = block_exscan(sy, wsum, btot);
#pragma unroll
    for (int j = 0; j < SUB_PER_T; j++) {
      const uint32_t sb = SUB_PER_T * tid + j;
      if (sb < nsub) { w.u_uniq_off[u0 + sb] = ex; w.u_bytes_off[u0 + sb] = ey; }
      ex += v[j];
      ey += y[j];
    }
    if (tid == 0) { w.b_uniq[b] = tot; w.b_bytes[b] = btot; }
  }
  // long-table slice b
  const uint64_t L = w.long_cap / NB, s0 = (uint64_t)b * L;
  if (tid == 0) { lsn = 0; lsb = 0; }
  __syncthreads();
  unsigned long long n = 0, by = 0;
  for (uint64_t i = tid; i < L; i += blockDim.x) {
    const LSlot e = w.ltab[s0 + i];
    if (e.h) { n++; by += e.len; }
  }
  if (n) { atomicAdd(&lsn, n); atomicAdd(&lsb, by); }
  __syncthreads();
  if (tid == 0) { w.ls_n[b] = lsn; w.ls_b[b] = lsb; }
}

// One workgroup of NB threads: partition / slice offsets, table sizes and the
// table-capacity checks.  Short words come first
// (partition order = hash order), then long words in slot order.
__device__ void final_scan(const Work& w) {
  __shared__ uint64_t wsum[16];
  const bool rerun = (w.ctl->overflow & OVF_RERUN) != 0;  // nothing was reduced
  const uint32_t b = threadIdx.x;
  uint64_t ns, sb, nl, lb;
  w.uniq_off[b] = block_exscan(rerun ? 0 : w.b_uniq[b], wsum, ns);
  w.bytes_off[b] = block_exscan(rerun ? 0 : w.b_bytes[b], wsum, sb);
  w.ls_off[b] = block_exscan(rerun ? 0 : w.ls_n[b], wsum, nl);
  w.ls_boff[b] = block_exscan(rerun ? 0 : w.ls_b[b], wsum, lb);
  if (b == 0) {
    w.uniq_off[NB] = ns;
    w.bytes_off[NB] = sb;
    w.ls_off[NB] = nl;
    w.ls_boff[NB] = lb;
    w.ctl->n_short = ns;
    w.ctl->short_bytes = sb;
    w.ctl->n_total = ns + nl;
    w.ctl->bytes_total = sb + lb;
    if (ns + nl > w.table_cap) atomicOr(&w.ctl->overflow, OVF_TABLE);
    else w.t_offs[ns + nl] = sb + lb;
    if (sb + lb > w.bytes_cap) atomicOr(&w.ctl->overflow, OVF_BYTES);
  }
}
extern "C" __global__ __launch_bounds__(1024) void k_unit_uniq_scan(Work w) { unit_uniq_scan(w); }
extern "C" __global__ __launch_bounds__(NB) void k_final_scan(Work w) { final_scan(w); }  // one workgroup

// True when this attempt produced a complete table that fits its buffers.
__device__ __forceinline__ bool table_ok(const Work& w) {
  return !(w.ctl->overflow & (OVF_RERUN | OVF_TABLE | OVF_BYTES));
}

// Exclusive scan over a 256-thread workgroup of two values at once.
__device__ __forceinline__ void exscan2_256(uint32_t a, uint32_t b, uint32_t (*ws)[2], uint32_t& ea, uint32_t& eb,
                                            uint32_t& ta, uint32_t& tb) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const uint32_t ia = wave_incl_scan(a), ib = wave_incl_scan(b);
  if (lane == 63) { ws[wv][0] = ia; ws[wv][1] = ib; }
  lds_barrier();  // LDS-only barriers: global loads in flight stay in flight
  uint32_t pa = 0, pb = 0;
  ta = 0; tb = 0;
  for (int k = 0; k < 4; k++) { if (k < wv) { pa += ws[k][0]; pb += ws[k][1]; } ta += ws[k][0]; tb += ws[k][1]; }
  lds_barrier();
  ea = pa + ia - a;
  eb = pb + ib - b;
}

// k_mat (256-thread workgroups): the dense table in one pass -- counts, byte
// offsets and bytes of every short word, then of every long word, and lpos for
// the exchange pack.
//  * short words: a whole partition by one workgroup, each unit of a split
//    partition by one wave (no workgroup barrier).  Either way a step covers
//    a run of words (lane or thread = word): a scan of the key lengths gives the byte offsets, the
//    step's key bytes are assembled in LDS at their offset from the 16-byte
//    line below the step's first byte and written with aligned 16-byte
//    stores; bytes of the partial first and last lines (shared with the
//    neighbouring steps / units) are stored one by one;
//  * long words: long-table slice b by workgroup b (scan of the occupied
//    slots), after every wave of the workgroup is done with its units.
constexpr int MAT_WAVES = 4;
// Writes the staged bytes of [boff, boff + tot) (stage = LDS image of the
// 16-byte lines from gbase = boff & ~15) by `nt` threads with thread index t.
__device__ __forceinline__ void mat_flush(const Work& w, const uint8_t* st, uint64_t boff, uint64_t tot, uint32_t t,
                                          uint32_t nt) {
  const uint64_t gbase = boff & ~15ull, ge = boff + tot;
  const uint64_t a0 = (boff + 15) & ~15ull, a1 = ge & ~15ull;  // whole lines [a0, a1)
  if (a0 < a1) {
    for (uint64_t q = a0 + 16ull * t; q < a1; q += 16ull * nt)
      *reinterpret_cast<uint4*>(w.t_bytes + q) = *reinterpret_cast<const uint4*>(st + (q - gbase));
    if (t < 16 && boff + t < a0) w.t_bytes[boff + t] = st[(boff - gbase) + t];
    if (t >= 16 && t < 32 && a1 + (t - 16) < ge) w.t_bytes[a1 + (t - 16)] = st[(a1 - gbase) + (t - 16)];
  } else if (t < 32 && boff + t < ge) {
    w.t_bytes[boff + t] = st[(boff - gbase) + t];
  }
}
// One word of a step: its count, offset and (staged) bytes.  The stage is
// zeroed first and each key is OR-ed in as 5 byte-shifted dwords (its zero
// padding ORs nothing into the next word's bytes): 5 LDS atomics instead of
// one byte store per key byte.
__device__ __forceinline__ void mat_word(const Work& w, uint8_t* st, uint64_t dst, uint64_t boff, uint32_t ex, uint4 k,
                                         uint32_t len, unsigned long long cnt) {
  if (!MOX_CHK(w, dst < w.table_cap && boff + ex + len <= w.bytes_cap, CHK_MAT_ROW)) return;
  w.t_counts[dst] = cnt;
  w.t_offs[dst] = boff + ex;
  const uint32_t o = (uint32_t)(boff & 15ull) + ex, r = o & 3u;
  uint32_t* d = reinterpret_cast<uint32_t*>(st) + (o >> 2);
  const uint32_t kw[5] = {0u, k.x, k.y, k.z, k.w};
#pragma unroll
  for (int j = 0; j < 4; j++) {
    const uint32_t x = (uint32_t)((((uint64_t)kw[j + 1] << 32) | kw[j]) >> (32 - 8 * r));
    if (x) atomicOr(&d[j], x);
  }
  if (r && k.w >> (32 - 8 * r)) atomicOr(&d[4], k.w >> (32 - 8 * r));
}
// Zeroes stage bytes [0, n) (n a multiple of 16) with `nt` threads.
__device__ __forceinline__ void stage_zero(uint8_t* st, uint32_t n, uint32_t t, uint32_t nt) {
  for (uint32_t q = 16 * t; q < n; q += 16 * nt) *reinterpret_cast<uint4*>(st + q) = make_uint4(0, 0, 0, 0);
}
extern "C" __global__ __launch_bounds__(64 * MAT_WAVES) void k_mat(Work w, Corpus c) {
  __shared__ uint32_t ws[4][2];
  constexpr int WSTAGE = 64 * 16 + 32;  // one wave's step: 64 keys + the partial lines
  // per-wave stages; the workgroup path uses all of it as one 256-key stage
  __shared__ __attribute__((aligned(16))) uint8_t stage[MAT_WAVES * WSTAGE];
  static_assert(MAT_WAVES * WSTAGE >= 64 * MAT_WAVES * 16 + 32, "k_mat workgroup stage");
  if (!table_ok(w)) return;
  const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
  const uint32_t U = (uint32_t)w.ctl->n_units;
  // whole partitions (Zipf text: ~1,400 words each): workgroup b takes partition b
  for (uint32_t b = blockIdx.x; b < NB; b += gridDim.x) {
    // a whole partition is its own single unit: its key count (k_reduce), input
    // range and output offsets come straight from the partition directory
    const uint32_t kkb = w.b_kk[b];
    const uint64_t n = w.b_uniq[b], src0 = w.rec_off[b], dst0 = w.uniq_off[b];
    uint64_t boff = w.bytes_off[b];
    if (kkb != 0) continue;  // split: its units go to the waves below
    // one step = 256 words; the next step's words load while this one is
    // staged and written (LDS-only barriers keep those loads in flight)
    uint4 kn = make_uint4(0, 0, 0, 0);
    unsigned long long cn = 0;
    if ((uint64_t)tid < n) { kn = w.uk[src0 + tid]; cn = w.uc[src0 + tid]; }
    for (uint64_t i0 = 0; i0 < n; i0 += 64 * MAT_WAVES) {
      const uint64_t i = i0 + tid;
      const uint4 k = kn;
      const unsigned long long cnt = cn;
      const uint32_t len = i < n ? key_len16(k) : 0u;
      if (i + 64 * MAT_WAVES < n) { kn = w.uk[src0 + i + 64 * MAT_WAVES]; cn = w.uc[src0 + i + 64 * MAT_WAVES]; }
      stage_zero(stage, MAT_WAVES * WSTAGE, (uint32_t)tid, 64 * MAT_WAVES);
      uint32_t ex, dummy, tot, t2;
      exscan2_256(len, 0, ws, ex, dummy, tot, t2);  // its LDS barriers also order the zeroing
      if (i < n) mat_word(w, stage, dst0 + i, boff, ex, k, len, cnt);
      lds_barrier();
      mat_flush(w, stage, boff, tot, (uint32_t)tid, 64 * MAT_WAVES);
      lds_barrier();
      boff += tot;
    }
  }
  // units of split partitions (high-cardinality input: ~330 words each): one
  // wave each, up to 512 words per batch with all their loads issued at once
  // (count-1 units: the (index, count) pairs, then the key gathers from the
  // unit's split_k range)
  // words per lane per batch: 4 keeps k_mat at 76 VGPRs, 6 waves per SIMD (8:
  // 114 VGPRs, 4 waves; C4 16 GiB k_mat 12.1-12.4 -> 11.5-11.7 ms, g42)
  constexpr int MB = 4;
  for (uint32_t u = blockIdx.x * MAT_WAVES + wv; u < U; u += gridDim.x * MAT_WAVES) {
    const UnitDesc ud = w.udesc[u];
    if (ud.in_n == UNIT_WHOLE) continue;
    const uint64_t nf = w.u_uniq[u], n = nf & ~U_IDX;
    const bool byidx = (nf & U_IDX) != 0;  // count-1 unit: (record index, count) pairs
    const uint64_t src0 = ud.rec_off, dst0 = w.uniq_off[ud.part] + w.u_uniq_off[u];
    uint64_t boff = w.bytes_off[ud.part] + w.u_bytes_off[u];
    uint8_t* st = stage + wv * WSTAGE;
    for (uint64_t c0 = 0; c0 < n; c0 += 64 * MB) {
      uint4 kb[MB];
      unsigned long long cb[MB];
      if (byidx) {
        uint32_t v[MB];
#pragma unroll
        for (int s = 0; s < MB; s++) {
          const uint64_t i = c0 + s * 64 + lane;
          v[s] = i < n ? w.ui[src0 + i] : 0u;
        }
#pragma unroll
        for (int s = 0; s < MB; s++) {
          const uint64_t i = c0 + s * 64 + lane;
          kb[s] = i < n ? w.split_k[ud.in_off + (v[s] >> 16)] : make_uint4(0, 0, 0, 0);
          cb[s] = v[s] & 0xFFFFu;
        }
      } else {
#pragma unroll
        for (int s = 0; s < MB; s++) {
          const uint64_t i = c0 + s * 64 + lane;
          kb[s] = i < n ? w.uk[src0 + i] : make_uint4(0, 0, 0, 0);
          cb[s] = i < n ? w.uc[src0 + i] : 0ull;
        }
      }
#pragma unroll
      for (int s = 0; s < MB; s++) {
        const uint64_t i0 = c0 + s * 64;
        if (i0 >= n) break;  // wave-uniform
        const uint64_t i = i0 + lane;
        const uint32_t len = i < n ? key_len16(kb[s]) : 0u;
        stage_zero(st, WSTAGE, (uint32_t)lane, 64);
        const uint32_t incl = wave_incl_scan(len);
        const uint32_t tot = (uint32_t)__builtin_amdgcn_readlane((int)incl, 63);
        wave_lds_fence();
        if (i < n) mat_word(w, st, dst0 + i, boff, incl - len, kb[s], len, cb[s]);
        wave_lds_fence();
        mat_flush(w, st, boff, tot, (uint32_t)lane, 64);
        wave_lds_fence();  // the stage is rewritten by the next step
        boff += tot;
      }
    }
  }
  __syncthreads();
  // long words: slice b = slots [b L, (b + 1) L), in slot order
  const uint64_t ns = w.ctl->n_short, sb = w.ctl->short_bytes, L = w.long_cap / NB;
  for (uint32_t b = blockIdx.x; b < NB; b += gridDim.x) {
    if (w.ls_n[b] == 0) continue;
    uint64_t idx = w.ls_off[b], boff = sb + w.ls_boff[b];
    for (uint64_t i0 = 0; i0 < L; i0 += 256) {
      const uint64_t sl = (uint64_t)b * L + i0 + tid;
      LSlot e{};
      if (i0 + tid < L) e = w.ltab[sl];
      const uint32_t occ = e.h ? 1u : 0u;
      const uint32_t len = e.h ? (uint32_t)e.len : 0u;  // long words < 4 GiB
      uint32_t ei, eb, ti, tb;
      exscan2_256(occ, len, ws, ei, eb, ti, tb);
      if (occ) {
        const uint64_t di = ns + idx + ei, o = boff + eb;
        w.lpos[sl] = idx + ei;
        w.t_counts[di] = e.count;
        w.t_offs[di] = o;
        const uint64_t ref = e.ref - 1;
        for (uint64_t j = 0; j < e.len; j++) w.t_bytes[o + j] = ref_byte(c.base, w.arena, ref, j);
      }
      idx += ti;
      boff += tb;
    }
  }
}

// ------------------------------------------------------------------ multi-GPU exchange
//   Input: this rank's dense table after a local run.  Short
// words travel as WRec (key, count) in dense order, which is partition order
// and therefore owner order (part_owner); long words as XHdr + bytes, grouped
// per owner by long_owner(FNV hash).

// xcnt[d] for every destination d (xcnt zeroed by the host).
extern "C" __global__ void k_xcount(Work w, uint32_t P, XCnt* xcnt) {
  if (blockIdx.x == 0 && threadIdx.x < P) {
    const uint32_t d = threadIdx.x;
    xcnt[d].n_short = w.uniq_off[owner_first_part(d + 1, P)] - w.uniq_off[owner_first_part(d, P)];
  }
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < w.long_cap; s += stride) {
    const LSlot e = w.ltab[s];
    if (!e.h) continue;
    const uint32_t d = long_owner(e.h, P);
    atomicAdd(&xcnt[d].n_long, 1ull);
    atomicAdd(&xcnt[d].long_bytes, (unsigned long long)((e.len + 7) & ~7ull));
  }
}

// Short words in dense order as WRec (same unit mapping as k_mat_counts).
extern "C" __global__ void k_xpack_short(Work w, WRec* out) {
  const uint32_t U = (uint32_t)w.ctl->n_units;
  for (uint32_t u = blockIdx.x; u < U; u += gridDim.x) {
    const UnitDesc ud = w.udesc[u];
    const uint64_t nf = w.u_uniq[u], n = nf & ~U_IDX, src0 = ud.rec_off, dst0 = w.uniq_off[ud.part] + w.u_uniq_off[u];
    for (uint64_t i = threadIdx.x; i < n; i += blockDim.x) {
      uint4 k;
      unsigned long long cnt;
      if (nf & U_IDX) {
        const uint32_t v = w.ui[src0 + i];
        k = w.split_k[ud.in_off + (v >> 16)];
        cnt = v & 0xFFFFu;
      } else {
        k = w.uk[src0 + i];
        cnt = w.uc[src0 + i];
      }
      out[dst0 + i] = WRec{((uint64_t)k.y << 32) | k.x, ((uint64_t)k.w << 32) | k.z, cnt};
    }
  }
}

// Long words into per-destination blobs [XHdr x n_long][bytes]; cur = 2P
// zeroed cursors (headers, bytes).  Bytes come from the materialised table.
extern "C" __global__ void k_xpack_long(Work w, XDir dir, unsigned long long* cur, uint8_t* blob) {
  const uint64_t ns = w.ctl->n_short;
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t s = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; s < w.long_cap; s += stride) {
    const LSlot e = w.ltab[s];
    if (!e.h) continue;
    const uint32_t d = long_owner(e.h, dir.P);
    const uint64_t k = atomicAdd(&cur[d], 1ull);
    const uint64_t bo = atomicAdd(&cur[dir.P + d], (unsigned long long)((e.len + 7) & ~7ull));
    const uint64_t i = ns + w.lpos[s];
    uint8_t* base = blob + dir.blob[d];
    reinterpret_cast<XHdr*>(base)[k] = XHdr{e.h, e.len, w.t_counts[i], bo};
    uint8_t* o = base + dir.nlong[d] * sizeof(XHdr) + bo;
    const uint8_t* src = w.t_bytes + w.t_offs[i];
    for (uint64_t j = 0; j < e.len; j++) o[j] = src[j];
  }
}

// Received partials -> reduce input.  Short WRecs are already in w.w (count in
// ctl->w_n); long words are inserted into the long table with arena refs (the
// received blob area was copied to the arena).  Sums all counts into
// ctl->tokens.
extern "C" __global__ void k_xingest(Work w, XDir dir, uint64_t n_short) {
  const uint64_t nlong = dir.hpre[dir.P];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  unsigned long long tok = 0;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n_short; t += stride) tok += w.w[t].count;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t < nlong; t += stride) {
    uint32_t a = 0, b = dir.P - 1;  // source s with hpre[s] <= t < hpre[s+1]
    while (a < b) { const uint32_t m = (a + b + 1) >> 1; if (dir.hpre[m] <= t) a = m; else b = m - 1; }
    const uint64_t base = dir.blob[a];
    const XHdr hd = reinterpret_cast<const XHdr*>(w.arena + base)[t - dir.hpre[a]];
    const uint64_t ref = base + dir.nlong[a] * sizeof(XHdr) + hd.off;
    long_insert(w, nullptr, hd.h, ARENA_BIT | ref, hd.len, hd.count);
    atomicAdd(&w.ctl->long_n, 1ull);
    tok += hd.count;
  }
  __shared__ unsigned long long s_tok;
  if (threadIdx.x == 0) s_tok = 0;
  __syncthreads();
  for (int off = 32; off > 0; off >>= 1) tok += __shfl_down(tok, off);
  if ((threadIdx.x & 63) == 0 && tok) atomicAdd(&s_tok, tok);
  __syncthreads();
  if (threadIdx.x == 0 && s_tok) atomicAdd(&w.ctl->tokens, s_tok);  // one global atomic per workgroup
}

// ---- sorted exchange (byte-range ownership; XSplit, mox_internal.h)
// Bytes [o, o + 16) of the table as two little-endian words, from aligned
// 8-byte loads and a funnel shift (t_bytes has 64 bytes of slack past its
// end: realloc_sized), instead of one load per byte.
__device__ __forceinline__ void table_bytes16(const Work& w, uint64_t o, uint64_t& k0, uint64_t& k1) {
  const uint64_t* q = reinterpret_cast<const uint64_t*>(w.t_bytes + (o & ~7ull));
  const uint32_t sh = (uint32_t)(o & 7u) * 8u;
  const uint64_t a = q[0], b = q[1], c = q[2];
  k0 = sh ? (a >> sh) | (b << (64 - sh)) : a;
  k1 = sh ? (b >> sh) | (c << (64 - sh)) : b;
}
__device__ __forceinline__ uint64_t mask_bytes(uint64_t x, uint64_t n) { return n >= 8 ? x : x & ((1ull << (8 * n)) - 1ull); }
// The first 8 bytes of table row i, big-endian, zero padded.
__device__ __forceinline__ uint64_t row_prefix(const Work& w, uint64_t i) {
  const uint64_t o = w.t_offs[i], len = w.t_offs[i + 1] - o;
  uint64_t k0, k1;
  table_bytes16(w, o, k0, k1);
  (void)k1;
  return __builtin_bswap64(mask_bytes(k0, len));
}
// This rank's sample block (XS_BLOCK words at out): XS_SAMPLES prefixes of its
// local table, evenly over its rows (the table is in hash order, so they are a
// uniform sample of its distinct words; XS_NONE for an empty table), sorted
// ascending by a bitonic sort in LDS, then the table size (their weight).
// One workgroup of XS_SAMPLES threads.
extern "C" __global__ __launch_bounds__(XS_SAMPLES) void k_xsample(Work w, uint64_t* out) {
  __shared__ uint64_t v[XS_SAMPLES];
  const uint32_t t = threadIdx.x;
  const uint64_t n = w.ctl->n_total;
  v[t] = n ? row_prefix(w, (uint64_t)t * n / XS_SAMPLES) : XS_NONE;
  __syncthreads();
  for (uint32_t k = 2; k <= XS_SAMPLES; k <<= 1)
    for (uint32_t j = k >> 1; j > 0; j >>= 1) {
      const uint32_t l = t ^ j;
      uint64_t a = 0, b = 0;
      const bool act = l > t;
      if (act) { a = v[t]; b = v[l]; }
      __syncthreads();
      if (act && ((a > b) == ((t & k) == 0))) { v[t] = b; v[l] = a; }
      __syncthreads();
    }
  out[t] = v[t];
  if (t < XS_BLOCK - XS_SAMPLES) out[XS_SAMPLES + t] = t == 0 ? n : 0ull;
}

// Splitters of the sorted exchange from every rank's sample block (blocks:
// P x XS_BLOCK words, the same on every rank), on the device: no host round
// trip between the sample all-to-all and the counts.  Rank q's samples weigh
// n_q (its table size) each, so a rank with more words takes more of the
// ranges (equal weights let a small shard's samples set half the splitters).
// A value v's weighted rank interval is (lo(v), hi(v)] with lo = sum_q n_q
// #(samples of q < v) and hi with <=; splitter k (1 <= k < P) is the value whose
// interval holds t_k = k W / P, W = sum_q n_q S (S samples per rank): every
// candidate sample checks every k, and equal values write the same splitter.
// With more than XS_LDS samples in all, every (S_all / S)-th sample of each
// (sorted) block is used.  flag = 1 when one value's interval is wider than
// XS_SKEW_NUM / XS_SKEW_DEN fair shares (skewed prefixes: the host falls back
// to hash owners).  One workgroup of 1024 threads.
extern "C" __global__ __launch_bounds__(1024) void k_xsplit(const uint64_t* blocks, uint32_t P, uint64_t* sp, uint32_t* flag) {
  __shared__ uint64_t v[XS_LDS];
  __shared__ uint64_t wq[MAX_RANKS];
  const uint32_t t = threadIdx.x;
  const uint32_t S = XS_SAMPLES * P <= XS_LDS ? XS_SAMPLES : XS_LDS / P;  // samples per rank used (a power of two)
  const uint32_t stride = XS_SAMPLES / S;
  if (t < P) wq[t] = blocks[(uint64_t)t * XS_BLOCK + XS_SAMPLES];
  if (t + 1 < P) sp[t] = 0;
  if (t == 0) *flag = 0;
  for (uint32_t i = t; i < S * P; i += 1024) {
    const uint32_t q = i / S, j = i % S;
    v[i] = blocks[(uint64_t)q * XS_BLOCK + (uint64_t)j * stride];
  }
  __syncthreads();
  uint64_t W = 0;
  for (uint32_t q = 0; q < P; q++) W += wq[q] * S;
  if (W == 0) return;
  for (uint32_t i = t; i < S * P; i += 1024) {
    const uint64_t x = v[i];
    if (x == XS_NONE) continue;  // an empty table's samples (weight 0)
    uint64_t lo = 0, hi = 0;
    for (uint32_t q = 0; q < P; q++) {
      if (!wq[q]) continue;
      const uint64_t* b = v + (uint64_t)q * S;
      uint32_t a = 0, z = S;  // lower bound: first sample >= x
      while (a < z) { const uint32_t m = (a + z) >> 1; if (b[m] < x) a = m + 1; else z = m; }
      uint32_t a2 = a, z2 = S;  // upper bound: first sample > x
      while (a2 < z2) { const uint32_t m = (a2 + z2) >> 1; if (b[m] <= x) a2 = m + 1; else z2 = m; }
      lo += wq[q] * a;
      hi += wq[q] * a2;
    }
    for (uint32_t k = 1; k < P; k++) {
      const uint64_t tk = (uint64_t)k * W / P;  // (W <= 2^48: table rows < 2^32, S <= 2^10, P <= 2^6)
      if (lo < tk && tk <= hi) sp[k - 1] = x;
    }
    // skew: this value alone is more than XS_SKEW_NUM / XS_SKEW_DEN of W / P
    if (P > 1 && (hi - lo) * P * XS_SKEW_DEN > W * XS_SKEW_NUM) *flag = 1;
  }
}
// Rows of the local table per block: a contiguous chunk each
constexpr uint32_t XR_THREADS = 256;
__device__ __forceinline__ void xr_chunk(uint64_t n, uint64_t& r0, uint64_t& r1) {
  const uint64_t per = (n + gridDim.x - 1) / gridDim.x;
  r0 = (uint64_t)blockIdx.x * per;
  r0 = r0 < n ? r0 : n;
  r1 = r0 + per < n ? r0 + per : n;
}
// Per-destination counts of the sorted exchange (xcnt zeroed by the host): short
// words (table rows < n_short) and long words (the rest), by range owner.  One
// global atomic per (workgroup, destination) for the short words.
extern "C" __global__ __launch_bounds__(XR_THREADS) void k_xcount_r(Work w, XSplit x, XCnt* xcnt) {
  __shared__ uint32_t lc[MAX_RANKS];
  __shared__ uint64_t sp[MAX_RANKS];
  const uint32_t t = threadIdx.x;
  if (t < MAX_RANKS) lc[t] = 0;
  if (t + 1 < x.P) sp[t] = x.sp[t];
  __syncthreads();
  const uint64_t ns = w.ctl->n_short, n = w.ctl->n_total;
  uint64_t r0, r1;
  xr_chunk(n, r0, r1);
  for (uint64_t i = r0 + t; i < r1; i += XR_THREADS) {
    const uint32_t d = range_owner(sp, x.P, row_prefix(w, i));
    if (i < ns) {
      atomicAdd(&lc[d], 1u);
    } else {
      atomicAdd(&xcnt[d].n_long, 1ull);
      atomicAdd(&xcnt[d].long_bytes, (unsigned long long)((w.t_offs[i + 1] - w.t_offs[i] + 7) & ~7ull));
    }
  }
  __syncthreads();
  if (t < x.P && lc[t]) atomicAdd(&xcnt[t].n_short, (unsigned long long)lc[t]);
}
// Pack of the sorted exchange: short words as WRec (key = the row's bytes, zero
// padded) at x.soff[d] + a range the workgroup reserves per destination
// (cur[d]); long words as XHdr + bytes into destination d's blob (cursors
// cur[P + d] headers, cur[2 P + d] bytes; their FNV-1a-64 hash recomputed from
// the bytes, as the map computed it).  cur: 3 P words zeroed by the host.  The
// order inside a destination is not the row order (the receiver's reduce does
// not depend on it).
extern "C" __global__ __launch_bounds__(XR_THREADS) void k_xpack_r(Work w, XSplit x, XDir dir, unsigned long long* cur,
                                                                 WRec* out, uint8_t* blob) {
  __shared__ uint32_t lc[MAX_RANKS];
  __shared__ unsigned long long lb[MAX_RANKS];
  __shared__ uint64_t sp[MAX_RANKS];
  const uint32_t t = threadIdx.x, P = x.P;
  if (t < MAX_RANKS) lc[t] = 0;
  if (t + 1 < P) sp[t] = x.sp[t];
  __syncthreads();
  const uint64_t ns = w.ctl->n_short, n = w.ctl->n_total;
  uint64_t r0, r1;
  xr_chunk(ns, r0, r1);  // short rows: counted, then written at the reserved ranges
  for (uint64_t i = r0 + t; i < r1; i += XR_THREADS) atomicAdd(&lc[range_owner(sp, P, row_prefix(w, i))], 1u);
  __syncthreads();
  if (t < P) {
    lb[t] = lc[t] ? x.soff[t] + atomicAdd(&cur[t], (unsigned long long)lc[t]) : 0ull;
    lc[t] = 0;
  }
  __syncthreads();
  for (uint64_t i = r0 + t; i < r1; i += XR_THREADS) {
    const uint64_t o = w.t_offs[i], len = w.t_offs[i + 1] - o;  // a short word: at most 16 bytes
    uint64_t k0, k1;
    table_bytes16(w, o, k0, k1);
    k0 = mask_bytes(k0, len);
    k1 = len > 8 ? mask_bytes(k1, len - 8) : 0ull;
    const uint64_t pre = __builtin_bswap64(k0);
    const uint32_t d = range_owner(sp, P, pre);
    const uint32_t r = atomicAdd(&lc[d], 1u);
    out[lb[d] + r] = WRec{k0, k1, w.t_counts[i]};
  }
  // long words (rare): one global atomic per word and cursor
  for (uint64_t i = ns + (uint64_t)blockIdx.x * XR_THREADS + t; i < n; i += (uint64_t)gridDim.x * XR_THREADS) {
    const uint64_t o = w.t_offs[i], len = w.t_offs[i + 1] - o;
    const uint32_t d = range_owner(sp, P, row_prefix(w, i));
    uint64_t h = FNV0;
    for (uint64_t j = 0; j < len; j++) h = fnv_step(h, w.t_bytes[o + j]);
    h = fnv_finish(h);
    const uint64_t k = atomicAdd(&cur[P + d], 1ull);
    const uint64_t bo = atomicAdd(&cur[2 * P + d], (unsigned long long)((len + 7) & ~7ull));
    uint8_t* base = blob + dir.blob[d];
    reinterpret_cast<XHdr*>(base)[k] = XHdr{h, len, w.t_counts[i], bo};
    uint8_t* ob = base + dir.nlong[d] * sizeof(XHdr) + bo;
    for (uint64_t j = 0; j < len; j++) ob[j] = w.t_bytes[o + j];
  }
}

// ------------------------------------------------------------------ gather
// Root of mox_gather: offsets of the concatenated table.  Row t of the
// gathered table belongs to source s with base_n[s] <= t < base_n[s + 1];
// its offset is the source's own offset plus the bytes of the sources before
// it.  Row N (the end) gets the total.
extern "C" __global__ void k_gather_offs(const uint8_t* recv, GDir d, uint64_t* out) {
  const uint64_t N = d.base_n[d.P];
  const uint64_t stride = (uint64_t)gridDim.x * blockDim.x;
  for (uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; t <= N; t += stride) {
    if (t == N) { out[N] = d.base_b_total; continue; }
    uint32_t a = 0, b = d.P - 1;  // last source with base_n[s] <= t
    while (a < b) { const uint32_t m = (a + b + 1) >> 1; if (d.base_n[m] <= t) a = m; else b = m - 1; }
    const uint64_t* offs = reinterpret_cast<const uint64_t*>(recv + d.roff[a]);
    out[t] = offs[t - d.base_n[a]] + d.base_b[a];
  }
}

}  // namespace mox
