// Host engine + C ABI (include/mox.h) of the MI355X word-count engine.
//
// Replaces the reference's hot section (/root/reference/src/main.rs:16-22:
// split_file -> map_phase -> reduce_phase) with one device pipeline per call:
//   corpus in HBM -> dictionary -> map (+shuffle write) -> lanes -> directory
//   -> bucket reduce -> dense table in HBM.
// No host round-trip inside the pipeline; one small control-block read at the
// end decides success, UTF-8 error, or a buffer-growth rerun.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "mox_host.h"
#include "mox_unicode_tables.h"

namespace mox_host {

thread_local std::string g_err;

int fail(int code, const char* fmt, ...) {
  char buf[512];
  va_list ap;
  va_start(ap, fmt);
  vsnprintf(buf, sizeof buf, fmt, ap);
  va_end(ap);
  g_err = buf;
  return code;
}


int dalloc(mox_engine* e, void** p, size_t bytes) {
  if (bytes == 0) bytes = 16;
  hipError_t err = hipMalloc(p, bytes);
  if (err != hipSuccess) return fail(MOX_ENOMEM, "hipMalloc(%zu) failed: %s", bytes, hipGetErrorString(err));
  return MOX_OK;
}
void dfree(void* p) {
  if (p) (void)hipFree(p);
}


Caps caps_of(const Work& w) {
  return Caps{w.cold_cap, w.spill_cap, w.w_cap, w.u_cap, w.arena_cap, w.long_cap, w.table_cap, w.bytes_cap, w.split_k_cap, w.split_w_cap};
}

Caps initial_caps(uint64_t n, int map_grid) {
  Caps c;
  // cold records per (workgroup, partition) region: about one per 8 input bytes
  c.cold_cap = std::max<uint64_t>(64, n / ((uint64_t)map_grid * NB * 8));
  c.spill_cap = std::max<uint64_t>(1024, n / ((uint64_t)map_grid * 64));
  c.w_cap = 65536 + n / 64;
  c.u_cap = 4096 + n / 64;
  c.arena_cap = 65536 + n / 16;
  c.long_cap = 65536;
  c.table_cap = 65536 + n / 64;
  c.bytes_cap = c.table_cap * 8;
  c.split_k_cap = 0;  // grown on demand (OVF_SPLIT): only high-cardinality inputs split partitions
  c.split_w_cap = 0;
  return c;
}

#define FREE_FIELD(f) \
  do {                \
    dfree(e->w.f);    \
    e->w.f = nullptr; \
  } while (0)

void free_sized(mox_engine* e) {
  FREE_FIELD(cold); FREE_FIELD(spill);
  FREE_FIELD(w); FREE_FIELD(w_sorted); FREE_FIELD(u); FREE_FIELD(arena); FREE_FIELD(ltab); FREE_FIELD(lpos);
  FREE_FIELD(uk); FREE_FIELD(uc); FREE_FIELD(ui); FREE_FIELD(t_counts); FREE_FIELD(t_offs); FREE_FIELD(t_bytes);
  FREE_FIELD(split_k); FREE_FIELD(split_w);
  Work& w = e->w;
  w.cold_cap = w.spill_cap = 0;
  w.w_cap = w.u_cap = w.arena_cap = w.long_cap = w.uniq_cap = w.table_cap = w.bytes_cap = 0;
  w.split_k_cap = w.split_w_cap = 0;
}

// Allocates every size-dependent buffer for capacities c.  The new capacities
// are committed to e->w only after every allocation succeeded: on a failure
// everything is freed and the capacities are zero (w.cold == nullptr), so the
// next ensure_caps reallocates instead of launching kernels on null buffers
// with a stale recorded capacity.
int realloc_sized(mox_engine* e, const Caps& c) {
  (void)hipDeviceSynchronize();
  free_sized(e);
  Work n = e->w;
  // a multiple of 2 QF_MAX: every one of a region's QF_MAX slices holds an even
  // number of records, so k_map's paired records stay sector-aligned
#ifndef MOX_COLD_PAD
#define MOX_COLD_PAD 0  // experiment: extra 2 QF_MAX-record steps per region (region stride off a power of two)
#endif
  n.cold_cap = (uint32_t)std::min<uint64_t>(((c.cold_cap + 2 * QF_MAX - 1) & ~(uint64_t)(2 * QF_MAX - 1)) + MOX_COLD_PAD * 2 * QF_MAX,
                                            COLD_CAP_MAX);
  static_assert(COLD_CAP_MAX % (2 * QF_MAX) == 0 && COLD_CAP_MAX < (1u << 24), "cold_cap clamp (k_map: __umul24)");
  n.spill_cap = (uint32_t)std::min<uint64_t>(c.spill_cap, 0xFFFFFFF0u);
  n.w_cap = c.w_cap;
  n.u_cap = c.u_cap;
  n.arena_cap = c.arena_cap;
  n.long_cap = next_pow2(c.long_cap);
  n.uniq_cap = (uint64_t)n.map_grid * NB * n.cold_cap + c.w_cap;
  n.table_cap = c.table_cap;
  n.bytes_cap = c.bytes_cap;
  n.split_k_cap = c.split_k_cap;
  n.split_w_cap = c.split_w_cap;
  struct { void** p; uint64_t bytes; } plan[] = {
      {(void**)&n.cold, (uint64_t)n.map_grid * NB * n.cold_cap * 16}, {(void**)&n.spill, (uint64_t)n.map_grid * n.spill_cap * 16},
      {(void**)&n.w, n.w_cap * sizeof(WRec)}, {(void**)&n.w_sorted, n.w_cap * sizeof(WRec)},
      {(void**)&n.u, n.u_cap * sizeof(URec)}, {(void**)&n.arena, n.arena_cap},
      {(void**)&n.ltab, n.long_cap * sizeof(LSlot)}, {(void**)&n.lpos, (n.long_cap + 1) * 8},
      {(void**)&n.uk, n.uniq_cap * 16}, {(void**)&n.uc, n.uniq_cap * 8}, {(void**)&n.ui, n.uniq_cap * 4},
      {(void**)&n.t_counts, n.table_cap * 8}, {(void**)&n.t_offs, (n.table_cap + 1) * 8},
      {(void**)&n.t_bytes, n.bytes_cap + 64}, {(void**)&n.split_k, n.split_k_cap * 16},  // (t_bytes: 64 B of slack for
                                                                                          // aligned 8-byte reads past a word)
      {(void**)&n.split_w, n.split_w_cap * sizeof(WRec)}};
  for (auto& a : plan) *a.p = nullptr;
  for (auto& a : plan) {
    int rc = (e->test_fail_alloc && --e->test_fail_alloc == 0)
                 ? fail(MOX_ENOMEM, "hipMalloc(%llu) failed: injected (MOX_TEST_FAIL_ALLOC)", (unsigned long long)a.bytes)
                 : dalloc(e, a.p, a.bytes);
    if (rc) {
      const std::string msg = g_err;
      for (auto& b : plan) dfree(*b.p);
      g_err = msg;
      return rc;  // e->w keeps null buffers and zero capacities
    }
  }
  e->w = n;
  return MOX_OK;
}

bool caps_cover(const Caps& have, const Caps& need) {
  return have.cold_cap >= need.cold_cap && have.spill_cap >= need.spill_cap && have.w_cap >= need.w_cap && have.u_cap >= need.u_cap &&
         have.arena_cap >= need.arena_cap && have.long_cap >= need.long_cap && have.table_cap >= need.table_cap &&
         have.bytes_cap >= need.bytes_cap && have.split_k_cap >= need.split_k_cap && have.split_w_cap >= need.split_w_cap;
}

Caps caps_max(const Caps& a, const Caps& b) {
  return Caps{std::max(a.cold_cap, b.cold_cap), std::max(a.spill_cap, b.spill_cap), std::max(a.w_cap, b.w_cap), std::max(a.u_cap, b.u_cap),
              std::max(a.arena_cap, b.arena_cap), std::max(a.long_cap, b.long_cap),
              std::max(a.table_cap, b.table_cap), std::max(a.bytes_cap, b.bytes_cap), std::max(a.split_k_cap, b.split_k_cap),
              std::max(a.split_w_cap, b.split_w_cap)};
}

int ensure_caps(mox_engine* e, const Caps& need) {
  if (e->w.cold && caps_cover(caps_of(e->w), need)) return MOX_OK;
  Caps c = e->w.cold ? caps_max(caps_of(e->w), need) : need;
  return realloc_sized(e, c);
}

// Dictionary buffer set i becomes the one the next enqueued kernels use.
void use_dset(mox_engine* e, int i) {
  const mox_engine::DictSet& d = e->dsets[i];
  e->w.cand = d.cand;
  e->w.dict_hist = d.dict_hist;
  e->w.dict_list = d.dict_list;
  e->w.dict_tag = d.dict_tag;
  e->w.dict_key = d.dict_key;
  e->w.dict_tot = d.dict_tot;
  e->dcur = i;
}

int alloc_fixed(mox_engine* e) {
  Work& w = e->w;
  int rc;
  if ((rc = dalloc(e, (void**)&w.ctl, sizeof(Ctl)))) return rc;
  for (auto& d : e->dsets) {  // two dictionary sets (async passes alternate, mox_host.h)
    if ((rc = dalloc(e, (void**)&d.cand, (size_t)GC_SLOTS * sizeof(WRec)))) return rc;
    if ((rc = dalloc(e, (void**)&d.dict_hist, 260 * 4))) return rc;  // 257 used, zeroed as 260 (k_init)
    if ((rc = dalloc(e, (void**)&d.dict_list, (size_t)DICT_MAX_WORDS * sizeof(WRec)))) return rc;
    if ((rc = dalloc(e, (void**)&d.dict_tag, DICT_SLOTS * 4))) return rc;
    if ((rc = dalloc(e, (void**)&d.dict_key, DICT_SLOTS * 16))) return rc;
    if ((rc = dalloc(e, (void**)&d.dict_tot, DICT_SLOTS * 8))) return rc;
    HIPCHK(hipMemset(d.dict_tag, 0, DICT_SLOTS * 4));
  }
  use_dset(e, 0);
  w.map_grid = (uint32_t)std::min(e->n_cu * MAP_WG_PER_CU, MAX_MAP_GRID);
  // region counters and split samples for up to QF_MAX regions per (map workgroup, partition)
  if ((rc = dalloc(e, (void**)&w.cold_n, (size_t)w.map_grid * NB * QF_MAX * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.samp, (size_t)w.map_grid * NB * QF_MAX * SPLIT_PER_REGION * 4))) return rc;
  HIPCHK(hipMemset(w.samp, 0, (size_t)w.map_grid * NB * QF_MAX * SPLIT_PER_REGION * 4));
  if ((rc = dalloc(e, (void**)&w.spill_n, (size_t)w.map_grid * 4))) return rc;
  // bucket directory block: one allocation, zeroed per run
  size_t dir_bytes = NB * 8 + NB * 4 + NB * 4 + 2 * (NB + 1) * 8 + NB * 8 + (NB + 1) * 8;
  uint8_t* d;
  if ((rc = dalloc(e, (void**)&d, dir_bytes))) return rc;
  w.b_recs = (uint64_t*)d; d += NB * 8;
  w.b_w = (uint32_t*)d; d += NB * 4;
  w.b_cur = (uint32_t*)d; d += NB * 4;
  w.w_off = (uint64_t*)d; d += (NB + 1) * 8;
  w.rec_off = (uint64_t*)d; d += (NB + 1) * 8;
  w.b_uniq = (uint64_t*)d; d += NB * 8;
  w.uniq_off = (uint64_t*)d; d += (NB + 1) * 8;
  // reduce units (high-cardinality split)
  if ((rc = dalloc(e, (void**)&w.b_kk, NB * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.red_order, NB * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.u_base, (NB + 1) * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.sub_hist, (size_t)NB * 2 * SUB_N * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.sp_off, (NB + 1) * 8))) return rc;
  if ((rc = dalloc(e, (void**)&w.spw_off, (NB + 1) * 8))) return rc;
  if ((rc = dalloc(e, (void**)&w.udesc, (size_t)U_MAX * sizeof(UnitDesc)))) return rc;
  if ((rc = dalloc(e, (void**)&w.big_units, (size_t)U_MAX * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.mid_units, (size_t)U_MAX * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.small_units, (size_t)U_MAX * 4))) return rc;
  if ((rc = dalloc(e, (void**)&w.u_bytes, (size_t)U_MAX * 8))) return rc;
  if ((rc = dalloc(e, (void**)&w.u_bytes_off, (size_t)U_MAX * 8))) return rc;
  {
    uint64_t* t2;
    if ((rc = dalloc(e, (void**)&t2, 6 * (NB + 1) * 8))) return rc;
    w.b_bytes = t2; t2 += NB + 1;
    w.bytes_off = t2; t2 += NB + 1;
    w.ls_n = t2; t2 += NB + 1;
    w.ls_b = t2; t2 += NB + 1;
    w.ls_off = t2; t2 += NB + 1;
    w.ls_boff = t2;
  }
  if ((rc = dalloc(e, (void**)&w.u_uniq, (size_t)U_MAX * 8))) return rc;
  if ((rc = dalloc(e, (void**)&w.u_uniq_off, (size_t)U_MAX * 8))) return rc;
  // Unicode tables
  size_t tb = (2 * MOX_LOWER_N + 2 * MOX_CASED_N + 2 * MOX_CI_N) * 4;
  uint32_t* t;
  if ((rc = dalloc(e, (void**)&t, tb))) return rc;
  uint32_t* p = t;
  HIPCHK(hipMemcpy(p, mox_lower_src, MOX_LOWER_N * 4, hipMemcpyHostToDevice)); e->tables.lower_src = p; p += MOX_LOWER_N;
  HIPCHK(hipMemcpy(p, mox_lower_dst, MOX_LOWER_N * 4, hipMemcpyHostToDevice)); e->tables.lower_dst = p; p += MOX_LOWER_N;
  HIPCHK(hipMemcpy(p, mox_cased_lo, MOX_CASED_N * 4, hipMemcpyHostToDevice)); e->tables.cased_lo = p; p += MOX_CASED_N;
  HIPCHK(hipMemcpy(p, mox_cased_hi, MOX_CASED_N * 4, hipMemcpyHostToDevice)); e->tables.cased_hi = p; p += MOX_CASED_N;
  HIPCHK(hipMemcpy(p, mox_ci_lo, MOX_CI_N * 4, hipMemcpyHostToDevice)); e->tables.ci_lo = p; p += MOX_CI_N;
  HIPCHK(hipMemcpy(p, mox_ci_hi, MOX_CI_N * 4, hipMemcpyHostToDevice)); e->tables.ci_hi = p; p += MOX_CI_N;
  e->tables.n_lower = MOX_LOWER_N;
  e->tables.n_cased = MOX_CASED_N;
  e->tables.n_ci = MOX_CI_N;
  HIPCHK(hipHostMalloc((void**)&e->h_ctl, sizeof(Ctl), hipHostMallocDefault));
  HIPCHK(hipHostMalloc((void**)&e->h_ctl_init, sizeof(Ctl), hipHostMallocDefault));
  memset(e->h_ctl_init, 0, sizeof(Ctl));
  e->h_ctl_init->err_utf8 = ~0ull;
  e->h_ctl_init->halo_err = ~0ull;
  return MOX_OK;
}

constexpr size_t map_lds_bytes() { return MAP_LDS_BYTES; }  // (mox_internal.h)
size_t reduce_lds_bytes() { return RED_LDS_BYTES; }

float ev_ms(mox_engine* e, int a, int b) {
  float ms = 0;
  if (hipEventElapsedTime(&ms, e->ev[a], e->ev[b]) != hipSuccess) return 0;
  return ms;
}

void Seq::rec(int i) const {  // map_only: events 1 and 2 (around k_map) only
  if ((i == 1 || i == 2) && map_ev[0]) {
    if (timing || map_only) (void)hipEventRecord(map_ev[i - 1], s);
    return;
  }
  if (timing || (map_only && (i == 1 || i == 2))) (void)hipEventRecord(e->ev[i], s);
}
void Seq::step(const char* name) const {
  if (!sync_each) return;
  hipError_t er = hipStreamSynchronize(s);
  fprintf(stderr, "[mox] %s done: %s\n", name, hipGetErrorString(er));
}

Seq seq_of(mox_engine* e) {
  const bool full = (e->flags & MOX_F_TIMING) != 0;
  return Seq{e, e->stream, full, e->sync_each, !full && (e->flags & MOX_F_TIMING_MAP) != 0};
}

// Stages 4-5 of a pass (shared by the corpus pass and the exchange pass):
// shuffle directory + bucket reduce, then the dense table.
void launch_reduce_tail(mox_engine* e, const Corpus& c, const Seq& q) {
  Work& w = e->w;
  hipStream_t s = e->stream;
  hipLaunchKernelGGL(k_hist, dim3(w.map_grid), dim3(1024), 0, s, w);  // last workgroup: partition offsets
  q.step("k_hist");
  hipLaunchKernelGGL(k_scatter, dim3(w.map_grid), dim3(1024), 0, s, w);
  q.step("k_scatter");
  hipLaunchKernelGGL(k_split_count, dim3(NB), dim3(256), 0, s, w);  // SC_THREADS
  q.step("k_split_count");
  hipLaunchKernelGGL(k_unit_scan, dim3(1), dim3(256), 0, s, w);  // SC_THREADS
  q.step("k_unit_scan");
  hipLaunchKernelGGL(k_split_scatter, dim3(NB), dim3(1024), 0, s, w);
  q.step("k_split_scatter");
  // count-1 small units first: its hash-collision fallbacks join k_reduce's work list
  hipLaunchKernelGGL(k_reduce_sort1, dim3(MOX_S1_WG * e->n_cu), dim3(256), 0, s, w);  // 4 waves per workgroup, one unit per wave
  q.step("k_reduce_sort1");
  hipLaunchKernelGGL(k_reduce_sort2, dim3(8 * e->n_cu), dim3(64), 0, s, w);  // one wave per unit of 513..1024 records
  q.step("k_reduce_sort2");
  hipLaunchKernelGGL(k_reduce, dim3(NB), dim3(RED_THREADS), reduce_lds_bytes(), s, w);  // workgroup b: partition b, then the work list
  q.step("k_reduce");
  hipLaunchKernelGGL(k_reduce_small, dim3(8 * e->n_cu), dim3(128), 0, s, w);  // persistent, 8 per CU (SR_THREADS)
  q.step("k_reduce_small");
  q.rec(4);
  hipLaunchKernelGGL(k_unit_uniq_scan, dim3(NB), dim3(1024), 0, s, w);
  q.step("k_unit_uniq_scan");
  hipLaunchKernelGGL(k_final_scan, dim3(1), dim3(NB), 0, s, w);
  q.step("k_final_scan");
  // 6 four-wave workgroups per CU (k_mat's occupancy), at least one per long-table slice
  hipLaunchKernelGGL(k_mat, dim3(std::max(NB, 6 * e->n_cu)), dim3(256), 0, s, w, c);
  q.step("k_mat");
  q.rec(5);
}

// Read the control block back and collect the phase timings.
int finish_pass(mox_engine* e, const Seq& q) {
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_ctl, e->w.ctl, sizeof(Ctl), hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (q.map_only && !q.sync_each) {
    e->stats.ms_dict = e->stats.ms_lanes = e->stats.ms_reduce = e->stats.ms_finalize = e->stats.ms_run = 0;
    e->stats.ms_map = ev_ms(e, 1, 2);
  }
  if (q.timing) {
    e->stats.ms_dict = ev_ms(e, 0, 1);
    e->stats.ms_map = ev_ms(e, 1, 2);
    e->stats.ms_lanes = ev_ms(e, 2, 3);
    e->stats.ms_reduce = ev_ms(e, 3, 4);
    e->stats.ms_finalize = ev_ms(e, 4, 5);
    e->stats.ms_run = ev_ms(e, 0, 5);
  }
  return MOX_OK;
}

// One attempt of the whole device pipeline.  Returns MOX_OK after the control
// block has been read back into e->h_ctl (caller inspects overflow / errors).
// Dictionary kernels of one pass on stream s.
void launch_dict(mox_engine* e, const Corpus& c, hipStream_t s, const Seq& q) {
  Work& w = e->w;
  hipLaunchKernelGGL(k_sample, dim3(e->sample_pieces), dim3(256), 0, s, c, w, e->sample_pieces);
  q.step("k_sample");
  hipLaunchKernelGGL(k_dict_hist, dim3(GC_SLOTS / 1024), dim3(1024), 0, s, w);
  q.step("k_dict_hist");
  hipLaunchKernelGGL(k_dict_pick, dim3(GC_SLOTS / 1024), dim3(1024), 0, s, w, e->dict_words);
  q.step("k_dict_pick");
  hipLaunchKernelGGL(k_dict_build, dim3(1), dim3(1024), 0, s, w, e->dict_words);
  q.step("k_dict_build");
}

// side: build the dictionary on e->dstream, overlapping the previous pass's
// reduce tail (async passes), in the dictionary set the previous pass did not
// use (mox_host.h dsets: no cross-stream wait on the previous pass).
void enqueue_pass(mox_engine* e, const Corpus& c, const Seq& q, bool side = false) {
  Work& w = e->w;
  hipStream_t s = e->stream;
  q.rec(0);
  const bool dict = !(e->flags & MOX_F_NO_DICT) && c.own_hi > c.own_lo;
  const bool sided = side && dict && !q.timing && !q.sync_each;
  // 1. hot dictionary from a sample
  if (sided) {
    use_dset(e, e->dcur ^ 1);
    // after the previous pass's k_map (ev_mapped): beside its reduce tail
    if (e->mapped_pending) (void)hipStreamWaitEvent(e->dstream, e->ev_mapped, 0);
    e->mapped_pending = false;
    hipLaunchKernelGGL(k_dict_zero, dim3(64), dim3(256), 0, e->dstream, w);
    launch_dict(e, c, e->dstream, q);
    (void)hipEventRecord(e->ev_dready, e->dstream);
  }
  // control block, partition counters, long table, sampling buffers: one launch
  hipLaunchKernelGGL(k_init, dim3(256), dim3(256), 0, s, w, 0ull, sided ? 4u : (dict ? 1u : 0u));  // INIT_DICT_SIDE / INIT_DICT
  q.step("k_init");
  if (sided) (void)hipStreamWaitEvent(s, e->ev_dready, 0);
  else if (dict) launch_dict(e, c, s, q);
  q.rec(1);
  // 2. map: one streaming pass over the corpus
  const uint64_t row0 = c.own_lo & ~15ull;
  const uint64_t nrows = c.own_hi > c.own_lo ? (c.own_hi - row0 + PAY - 1) / PAY : 0;
  const int grid = (int)w.map_grid;
  hipLaunchKernelGGL(k_map, dim3(grid), dim3(MAP_THREADS), map_lds_bytes(), s, c, w, nrows, 0u);
  q.step("k_map");
  q.rec(2);
#ifndef MOX_SIDE_AFTER_MAP
#define MOX_SIDE_AFTER_MAP 0  // 1: measured slower end to end (profiles/r05/c2_side_dict_overlap.txt)
#endif
  if (MOX_SIDE_AFTER_MAP && side && !q.timing && !q.sync_each) {  // the next async pass's side build waits for this k_map
    (void)hipEventRecord(e->ev_mapped, s);
    e->mapped_pending = true;
  }
  // 3. lanes
  hipLaunchKernelGGL(k_unicode, dim3(1024), dim3(256), 0, s, c, w, e->tables);  // + dictionary totals
  q.step("k_unicode");
  q.rec(3);
  // 4-5. shuffle directory + bucket reduce, table
  launch_reduce_tail(e, c, q);
}

int pipeline_once(mox_engine* e, const Corpus& c) {
  const Seq q = seq_of(e);
  enqueue_pass(e, c, q);
  return finish_pass(e, q);
}

// Region capacity that covers the largest region an attempt asked for
// (cold_need), bounded by 4x the mean tokens per region: every region is sized
// alike, so one skewed region (a hot word without a dictionary) would size all
// 262 K of them; beyond the bound its records spill (spill_cap grows instead).
uint64_t cold_cap_for(const mox_engine* e, const Ctl& h) {
  const uint64_t want = h.cold_need + h.cold_need / 8 + 16;
  const uint64_t bound = 4 * h.tokens / ((uint64_t)e->w.map_grid * NB) + 64;
  return std::min(want, std::max<uint64_t>(bound, e->w.cold_cap));
}

// Capacities that cover what an overflowed attempt asked for.
Caps grow_for(mox_engine* e, const Ctl& h) {
  Caps need = caps_of(e->w);
  if (h.overflow & OVF_POOL) {
    need.cold_cap = std::max<uint64_t>(need.cold_cap, cold_cap_for(e, h));
    need.spill_cap = std::max<uint64_t>(need.spill_cap, h.spill_need + h.spill_need / 4 + 1024);
  }
  if (h.overflow & OVF_W) {
    const uint64_t wn = std::max<uint64_t>(h.w_total, h.w_n);
    need.w_cap = std::max<uint64_t>(need.w_cap, wn + wn / 4 + 1024);
  }
  if (h.overflow & OVF_U) need.u_cap = h.u_n + h.u_n / 4 + 1024;
  if (h.overflow & OVF_ARENA) need.arena_cap = h.arena_n + h.arena_n / 4 + 65536;
  if (h.overflow & OVF_LONG) need.long_cap = next_pow2(2 * h.long_n + 1024);
  if (h.overflow & OVF_TABLE) need.table_cap = h.n_total + h.n_total / 4 + 1024;
  if (h.overflow & OVF_BYTES) need.bytes_cap = h.bytes_total + h.bytes_total / 4 + 65536;
  if (h.overflow & OVF_SPLIT) {
    uint64_t k = h.split_k + h.split_k / 8 + 4096, wv = h.split_w + h.split_w / 8 + 4096;
    // a second overflow: which partitions split is decided from a sample taken
    // anew by every attempt, so the asks can keep rising past an eighth; take
    // the bound every split layout fits in (each partition split at most into
    // SUB_N sub-buckets of even starts: split_span <= records + SUB_N + 1)
    if (need.split_k_cap || need.split_w_cap) {  // (the caps are 0 until the first OVF_SPLIT)
      k = std::max<uint64_t>(k, h.cold_recs + h.cold_recs / 8 + (uint64_t)NB * (SUB_N + 2));
      wv = std::max<uint64_t>(wv, h.w_total + h.w_total / 8 + 4096);
    }
    need.split_k_cap = std::max<uint64_t>(need.split_k_cap, k);
    need.split_w_cap = std::max<uint64_t>(need.split_w_cap, wv);
  }
  // a table overflow also means the byte estimate is stale
  if (h.overflow & OVF_TABLE) need.bytes_cap = std::max(need.bytes_cap, need.table_cap * 16);
  return need;
}

void commit_result(mox_engine* e, const Corpus& c, const Ctl& h);

// The table of the pass whose control block is h (in the t_* buffers) becomes
// the engine's result.
void set_result(mox_engine* e, const Ctl& h) {
  e->res.counts = e->w.t_counts;
  e->res.offs = e->w.t_offs;
  e->res.bytes = e->w.t_bytes;
  e->res.n = h.n_total;
  e->res.nb = h.bytes_total;
  e->res.tokens = h.tokens;
  e->res.pass = true;
  e->res.exchanged = false;
  e->res.sorted = false;
  e->have_result = true;
}

// Check builds (-DMOX_CHECK): a device bounds check failed during the pass
// (mox_internal.h, MOX_CHK).  Production builds never fail here.
int check_failed(const Ctl& h) {
  if (h.layout_err) return fail(MOX_EHIP, "k_map: dynamic LDS does not start at address 0 (static LDS in the kernel?)");
#ifdef MOX_CHECK
  if (h.dbg_cnt[0])
    return fail(MOX_EHIP, "device bounds check failed %llu times (largest site id %llu)", h.dbg_cnt[0], h.dbg_cnt[1]);
#else
  (void)h;
#endif
  return MOX_OK;
}

// Diagnostics builds only (-DMOX_ABLATE / -DMOX_STAMP, tools/): per-workgroup
// cycle stamps and the dictionary, written under $MOX_DEBUG_DIR (nothing is
// written without it).  Production builds compile none of this.
#if defined(MOX_ABLATE) || defined(MOX_STAMP)
FILE* debug_file(const char* name) {
  const char* dir = getenv("MOX_DEBUG_DIR");
  if (!dir) return nullptr;
  return fopen((std::string(dir) + "/" + name).c_str(), "w");
}
void debug_dump(mox_engine* e, const Ctl& h) {
  // k_reduce slow path: inserts, lane iterations not done, publication retries,
  // cold-stream slow lanes; red_try misses: two buckets full, publication
  // pending, same tag + other key, lost claim not resolved
  if (e->w.dbg & DBG_COUNT)
    fprintf(stderr, "mox dbg_cnt %llu %llu %llu %llu | %llu %llu %llu %llu\n", h.dbg_cnt[0], h.dbg_cnt[1], h.dbg_cnt[2],
            h.dbg_cnt[3], h.dbg_cnt[4], h.dbg_cnt[5], h.dbg_cnt[6], h.dbg_cnt[7]);
  if ((e->w.dbg & DBG_STAMP) && e->w.stamps) {
    std::vector<unsigned long long> st(8 * NB);
    (void)hipMemcpy(st.data(), e->w.stamps, st.size() * 8, hipMemcpyDeviceToHost);
    std::vector<unsigned long long> mc(8 * 1024 * MAP_WAVES);
    (void)hipMemcpy(mc.data(), e->w.stamps + 8 * 4096, mc.size() * 8, hipMemcpyDeviceToHost);
    FILE* g = debug_file("mapcyc.csv");
    if (g) {
      for (uint32_t i = 0; i < e->w.map_grid * MAP_WAVES; i++)
        fprintf(g, "%u,%llu,%llu,%llu,%llu,%llu,%llu,%llu\n", i, mc[8 * i], mc[8 * i + 1], mc[8 * i + 2], mc[8 * i + 3], mc[8 * i + 4],
                mc[8 * i + 5], mc[8 * i + 6]);
      fclose(g);
    }
    std::vector<unsigned long long> rc(4 * 1024 * 16);
    (void)hipMemcpy(rc.data(), e->w.stamps + 8 * 4096 + 8 * 1024 * MAP_WAVES, rc.size() * 8, hipMemcpyDeviceToHost);
    if (FILE* r = debug_file("redcyc.csv")) {
      for (size_t i = 0; i < rc.size() / 4; i++) fprintf(r, "%zu,%llu,%llu,%llu,%llu\n", i, rc[4 * i], rc[4 * i + 1], rc[4 * i + 2], rc[4 * i + 3]);
      fclose(r);
    }
    FILE* f = debug_file("stamps.csv");
    if (f) {
      for (int i = 0; i < NB; i++)
        fprintf(f, "%d,%llu,%llu,%llu,%llu,%llu,%llu,%llu\n", i, st[8 * i], st[8 * i + 1], st[8 * i + 2], st[8 * i + 3], st[8 * i + 4], st[8 * i + 5], st[8 * i + 6]);
      fclose(f);
    }
  }
  if (getenv("MOX_DUMP_DICT")) {
    std::vector<uint4> dk(DICT_SLOTS);
    std::vector<uint32_t> dt(DICT_SLOTS);
    std::vector<unsigned long long> tot(DICT_SLOTS);
    (void)hipMemcpy(dk.data(), e->w.dict_key, DICT_SLOTS * 16, hipMemcpyDeviceToHost);
    (void)hipMemcpy(dt.data(), e->w.dict_tag, DICT_SLOTS * 4, hipMemcpyDeviceToHost);
    (void)hipMemcpy(tot.data(), e->w.dict_tot, DICT_SLOTS * 8, hipMemcpyDeviceToHost);
    std::vector<int> order;
    unsigned long long sum = 0;
    for (int i = 0; i < DICT_SLOTS; i++) if (dt[i]) { order.push_back(i); sum += tot[i]; }
    std::sort(order.begin(), order.end(), [&](int a, int b) { return tot[a] > tot[b]; });
    fprintf(stderr, "[mox] dict words %zu, hits %llu of %llu tokens\n", order.size(), sum, (unsigned long long)h.tokens);
    {
      std::vector<WRec> cand(GC_SLOTS), lst(DICT_MAX_WORDS);
      std::vector<uint32_t> hist(257);
      (void)hipMemcpy(cand.data(), e->w.cand, GC_SLOTS * sizeof(WRec), hipMemcpyDeviceToHost);
      (void)hipMemcpy(lst.data(), e->w.dict_list, DICT_MAX_WORDS * sizeof(WRec), hipMemcpyDeviceToHost);
      (void)hipMemcpy(hist.data(), e->w.dict_hist, 257 * 4, hipMemcpyDeviceToHost);
      size_t nc = 0, ns = 0;
      uint64_t best = 0;
      for (auto& r : cand) if (r.count) { nc++; if ((r.w1 & ~(1ull << 63)) == 0) { ns++; best = std::max(best, (uint64_t)r.count); } }
      fprintf(stderr, "[mox] cand: %zu used, %zu with w1==0 (max count %llu); picked %u, thresh %u, hist[255]=%u hist[2]=%u\n", nc, ns,
              (unsigned long long)best, hist[256], h.dict_thresh, hist[255], hist[2]);
      int k = 0;
      for (uint32_t i = 0; i < std::min<uint32_t>(hist[256], DICT_MAX_WORDS) && k < 5; i++)
        if (lst[i].w1 == 0) { char b[9] = {0}; memcpy(b, &lst[i].w0, 8); fprintf(stderr, "[mox]   list short '%s' count %llu\n", b, (unsigned long long)lst[i].count); k++; }
    }
    int nshort = 0;
    for (size_t j = 0; j < order.size(); j++) {
      const int i = order[j];
      char wbuf[17] = {0};
      memcpy(wbuf, &dk[i], 16);
      if (strlen(wbuf) <= 4 && nshort < 6) { fprintf(stderr, "[mox]   short slot %d total %llu key '%s' tag %08x\n", i, tot[i], wbuf, dt[i]); nshort++; }
    }
    for (size_t j = 0; j < order.size() && j < 8; j++) {
      const int i = order[j];
      char wbuf[17] = {0};
      memcpy(wbuf, &dk[i], 16);
      fprintf(stderr, "[mox]   slot %d tag %08x total %llu key '%s'\n", i, dt[i], tot[i], wbuf);
    }
  }
}
#endif

int run_corpus(mox_engine* e, const Corpus& c) {
  if (e->dstream) HIPCHK(hipStreamSynchronize(e->dstream));  // no side-stream dictionary build in flight
  e->have_result = false;
  uint64_t n = c.own_hi - c.own_lo;
  Caps want = caps_max(initial_caps(n, e->n_cu), e->grow_hint);
  want.cold_cap = std::max<uint64_t>(want.cold_cap, e->next_cold_cap);
  int rc = ensure_caps(e, want);
  if (rc) return rc;
  e->grow_hint = Caps{};
  e->stats.retries = 0;
  for (int attempt = 0;; attempt++) {
    if ((rc = pipeline_once(e, c))) return rc;
    const Ctl& h = *e->h_ctl;
    if (e->verbose)
      fprintf(stderr, "[mox] attempt %d: overflow 0x%x cold_need %llu spill_need %llu w_total %llu u_n %llu n_total %llu caps cold %u spill %u w %llu run %.3f ms; units %llu, sort2 list %llu, k_reduce list %llu, split partitions %u, max sub-passes %u\n",
              attempt, h.overflow, h.cold_need, h.spill_need, h.w_total, h.u_n, h.n_total, e->w.cold_cap, e->w.spill_cap,
              (unsigned long long)e->w.w_cap, e->stats.ms_run, h.n_units, h.n_mid, h.n_big, h.n_split, h.max_sub);
#if defined(MOX_ABLATE) || defined(MOX_STAMP)
    debug_dump(e, h);
#endif
    if ((rc = check_failed(h))) return rc;
    if (h.err_utf8 != ~0ull) return fail(MOX_EUTF8, "stream did not contain valid UTF-8 (byte %llu)", h.err_utf8);
    if (h.halo_err != ~0ull)
      return fail(MOX_EHALO, "token at byte %llu runs past the end of a non-final shard buffer", h.halo_err);
    if (!h.overflow) break;
    if (h.overflow & OVF_REDUCE)
      return fail(MOX_ENOMEM, "a reduce partition holds more distinct words than it can split by hash");
    if (attempt >= GROW_RETRIES) return fail(MOX_ENOMEM, "buffer growth did not converge (overflow mask 0x%x)", h.overflow);
    Caps need = grow_for(e, h);
    e->stats.retries++;
    if ((rc = ensure_caps(e, need))) return rc;
  }
  commit_result(e, c, *e->h_ctl);
  return MOX_OK;
}

// The pass over c finished with control block h (no overflow, no error): its
// table is the engine's result.
void commit_result(mox_engine* e, const Corpus& c, const Ctl& h) {
  if (&h != e->h_ctl) std::memcpy(e->h_ctl, &h, sizeof(Ctl));  // an async pass: fetch reads e->h_ctl
  // spills are correct but slow (atomic scatter): size the regions for the
  // next run of this engine from what this one needed
  // (applied at the start of the next run: the buffers hold this run's table)
  if (h.spill_need) e->next_cold_cap = std::max<uint64_t>(e->next_cold_cap, cold_cap_for(e, h));
  e->stats.bytes = c.own_hi - c.own_lo;
  e->stats.tokens = h.tokens;
  e->stats.uniques = h.n_total;
  e->stats.dict_words = h.dict_n;
  e->stats.cold_records = h.cold_recs;
  e->stats.weighted_records = h.w_n;
  e->stats.unicode_tokens = h.u_n;
  e->stats.long_tokens = h.long_n;
  e->stats.chunks = h.cold_need;
  e->stats.max_subpasses = h.max_sub ? h.max_sub : 1;
  e->stats.reduce_units = h.n_units;
  e->stats.split_partitions = h.n_split;
  static_assert(sizeof(e->stats.path_hits) == sizeof(h.paths), "path counters");
  std::memcpy(e->stats.path_hits, h.paths, sizeof h.paths);
  e->last_corpus = c;
  set_result(e, h);
}

// ---- asynchronous passes (mox_run_range_async / mox_run_wait)
// Completes async slot k: waits for its control block, then either commits its
// result, or (overflow) re-runs its corpus synchronously with grown buffers --
// unless a later pass is already queued behind it, which supersedes it.
int complete_async(mox_engine* e, int k) {
  auto& a = e->aslot[k];
  if (!a.pending) return MOX_OK;
  a.pending = false;
  HIPCHK(hipEventSynchronize(a.ev_done));
  const Ctl& h = *a.h_ctl;
  auto& later = e->aslot[k ^ 1];
  if (int rc = check_failed(h)) return rc;
  if (h.err_utf8 != ~0ull) return fail(MOX_EUTF8, "stream did not contain valid UTF-8 (byte %llu)", h.err_utf8);
  if (h.halo_err != ~0ull)
    return fail(MOX_EHALO, "token at byte %llu runs past the end of a non-final shard buffer", h.halo_err);
  if (!h.overflow) {
    const bool map_only = (e->flags & (MOX_F_TIMING | MOX_F_TIMING_MAP)) != 0;
    if (map_only) {
      float ms = 0;
      if (hipEventElapsedTime(&ms, a.ev_map0, a.ev_map1) == hipSuccess) e->stats.ms_map = ms;
    }
    e->stats.retries = 0;
    commit_result(e, a.c, h);
    if (later.pending) e->have_result = false;  // the later pass is overwriting this table
    return MOX_OK;
  }
  if (later.pending) {
    // A later pass is queued behind this one: it ran after this one on the same
    // stream and overwrites this pass's table, so this one's result can never
    // be observed.  It is not re-run: the capacities it asked for
    // are remembered for the next run, and the later pass completes on its own
    // (re-run there only if it overflowed itself).
    e->grow_hint = caps_max(e->grow_hint, grow_for(e, h));
    e->stats.async_dropped++;
    return MOX_OK;
  }
  // overflowed: drain, then the synchronous path (retry loop)
  HIPCHK(hipStreamSynchronize(e->stream));
  if (e->dstream) HIPCHK(hipStreamSynchronize(e->dstream));
  e->stats.async_reruns++;
  return run_corpus(e, a.c);
}

int drain_async(mox_engine* e) {
  // the older pending slot first
  const int first = e->anext;  // slot written least recently
  int rc = complete_async(e, first);
  const int rc2 = complete_async(e, first ^ 1);
  if (e->dstream) HIPCHK(hipStreamSynchronize(e->dstream));
  return rc ? rc : rc2;
}

// Internal coordinates: c.base is the buffer address rounded down to 16 B,
// minus 16, so that every valid byte sits at >= 16 and a row's context lane
// (16 bytes before its payload) never underflows.  Loads clamp to
// [lo, hi), so nothing below the buffer is ever read.
Corpus make_corpus(const void* d_buf, size_t buf_len, size_t own_begin, size_t own_end, int at_end) {
  uintptr_t addr = (uintptr_t)d_buf;
  uint64_t mis = (addr & 15) + 16;
  Corpus c{};
  c.base = (const uint8_t*)(addr - mis);
  c.lo = mis;
  c.hi = mis + buf_len;
  c.own_lo = mis + own_begin;
  c.own_hi = mis + own_end;
  c.ctx_lo = mis;
  c.at_end = at_end ? 1 : 0;
  return c;
}


// One engine on HIP device dev (-1: the current device).
int engine_create_one(const mox_config* cfg, int dev, mox_engine** out) {
  *out = nullptr;
  mox_engine* e = new (std::nothrow) mox_engine();
  if (!e) return fail(MOX_ENOMEM, "host allocation failed");
  if (cfg) {
    e->flags = cfg->flags;
    if (cfg->dict_words) e->dict_words = std::min<uint32_t>(cfg->dict_words, DICT_MAX_WORDS);
    if (cfg->sample_pieces) e->sample_pieces = std::min<uint32_t>(cfg->sample_pieces, MAX_SAMPLE_PIECES);
  }
  int ndev = 0;
  if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) {
    delete e;
    return fail(MOX_EHIP, "no HIP device available");
  }
  if (dev < 0) {
    if (hipGetDevice(&dev) != hipSuccess) dev = 0;
  }
  if (dev >= ndev) {
    delete e;
    return fail(MOX_EINVAL, "device %d out of range (%d devices)", dev, ndev);
  }
  e->device = dev;
  hipError_t herr = hipSetDevice(dev);
  if (herr != hipSuccess) { delete e; return fail(MOX_EHIP, "hipSetDevice: %s", hipGetErrorString(herr)); }
  hipDeviceProp_t prop;
  if (hipGetDeviceProperties(&prop, dev) == hipSuccess) e->n_cu = prop.multiProcessorCount;
  if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
    delete e;
    return fail(MOX_EHIP, "hipStreamCreate failed");
  }
  for (auto& ev : e->ev) (void)hipEventCreate(&ev);
  if (hipStreamCreateWithFlags(&e->dstream, hipStreamNonBlocking) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_dready, hipEventDisableTiming) != hipSuccess ||
      hipEventCreateWithFlags(&e->ev_mapped, hipEventDisableTiming) != hipSuccess) {
    mox_engine_destroy(e);
    return fail(MOX_EHIP, "side stream / events: creation failed");
  }
  if (hipFuncSetAttribute((const void*)k_map, hipFuncAttributeMaxDynamicSharedMemorySize, (int)map_lds_bytes()) != hipSuccess ||
      hipFuncSetAttribute((const void*)k_reduce, hipFuncAttributeMaxDynamicSharedMemorySize, (int)reduce_lds_bytes()) != hipSuccess) {
    mox_engine_destroy(e);
    return fail(MOX_EHIP, "hipFuncSetAttribute(dynamic LDS) failed");
  }
  if (const char* d = getenv("MOX_DBG")) e->w.dbg = (uint32_t)strtoul(d, nullptr, 0);
  if (e->w.dbg & DBG_STAMP) (void)hipMalloc((void**)&e->w.stamps, 8 * 8 * 4096 + 8 * 8 * 1024 * MAP_WAVES + 8 * 4 * 1024 * 16);
  e->sync_each = getenv("MOX_SYNC_EACH") != nullptr;
  e->verbose = getenv("MOX_VERBOSE") != nullptr;
  if (const char* f = getenv("MOX_TEST_FAIL_ALLOC")) e->test_fail_alloc = atoi(f);
  int rc = alloc_fixed(e);
  if (rc == MOX_OK && cfg && cfg->reserve_bytes) rc = ensure_caps(e, initial_caps(cfg->reserve_bytes, e->n_cu));
  if (rc != MOX_OK) {
    std::string msg = g_err;
    mox_engine_destroy(e);
    g_err = msg;
    return rc;
  }
  *out = e;
  return MOX_OK;
}

// Host buffer -> the engine's corpus staging buffer d_text.
int stage_host_range(mox_engine* e, const uint8_t* text, size_t len) {
  if (len > e->d_text_cap) {
    dfree(e->d_text);
    e->d_text = nullptr;
    e->d_text_cap = 0;
    int rc = dalloc(e, (void**)&e->d_text, len + 64);
    if (rc) return rc;
    e->d_text_cap = len;
  }
  const bool timing = (e->flags & MOX_F_TIMING) != 0;
  if (timing) HIPCHK(hipEventRecord(e->ev[8], e->stream));
  if (len) HIPCHK(hipMemcpyAsync(e->d_text, text, len, hipMemcpyHostToDevice, e->stream));
  if (timing) HIPCHK(hipEventRecord(e->ev[9], e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (timing) e->stats.ms_h2d = ev_ms(e, 8, 9);
  return MOX_OK;
}


// File -> HBM: FILE_READERS threads each pread their
// chunks (c = t, t + FILE_READERS, ...) into two pinned buffers of their own and
// copy them with hipMemcpyAsync, so the page-cache / disk reads of one chunk
// overlap the PCIe copies of the others.  All copies go to ONE stream (one DMA
// queue): on the GPU box one stream moves 55 GB/s of pinned H2D copies and two
// or more streams 47-53 GB/s, while 8 pread threads alone read 73 GB/s from the
// page cache (profiles/r03_ingest_probe.txt), so per-reader streams left the
// pipeline at 40-44 GB/s.  A reader refills a buffer once the event recorded
// after its copy has completed.  Pinned buffers, stream and events are
// engine-owned and reused across calls.
constexpr int MAX_FILE_READERS = 16;
// Reader threads and chunk size of mox_count_file: MOX_FILE_READERS (1..16,
// default 8) and MOX_FILE_CHUNK_MIB (default 32) tune them; MOX_FILE_STREAMS=0
// gives every reader its own copy stream (the round-2 scheme, for A/B:
// tools/ingest_bench.py).
int file_readers() {
  static const int n = [] {
    const char* v = getenv("MOX_FILE_READERS");
    const int k = v ? atoi(v) : 8;
    return k < 1 ? 1 : (k > MAX_FILE_READERS ? MAX_FILE_READERS : k);
  }();
  return n;
}
bool file_shared_stream() {
  static const bool one = [] {
    const char* v = getenv("MOX_FILE_STREAMS");
    return !(v && atoi(v) == 0);
  }();
  return one;
}
size_t file_chunk() {
  static const size_t c = [] {
    const char* v = getenv("MOX_FILE_CHUNK_MIB");
    const long k = v ? atol(v) : 32;
    return (size_t)(k < 1 ? 1 : (k > 256 ? 256 : k)) << 20;
  }();
  return c;
}
// Bytes [off0, off0 + len) of a file -> d_text[0, len), by reader threads.
// start() launches them; wait_bytes(b) blocks until the copies of the first b
// bytes are enqueued (shared copy stream: an event recorded there afterwards
// completes once they have landed); finish() joins them and waits for the
// copies.  The destructor joins readers still running (an error path).
struct FileStager {
  mox_engine* e;
  int fd;
  uint64_t off0;
  size_t len, chunk = 0, nchunks = 0;
  int readers = 0;
  bool shared = true;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<char> issued;
  size_t prefix = 0;               // chunks 0 .. prefix - 1 enqueued
  std::atomic<bool> failed{false};
  std::vector<int> err;
  std::vector<std::string> msg;
  std::vector<std::thread> th;
  std::chrono::steady_clock::time_point t0;

  FileStager(mox_engine* e_, int fd_, uint64_t off0_, size_t len_) : e(e_), fd(fd_), off0(off0_), len(len_) {}
  ~FileStager() { for (auto& x : th) if (x.joinable()) { failed = true; x.join(); } }
  hipStream_t copy_stream() const { return e->file_stream[0]; }

  int start() {
    if (len > e->d_text_cap) {
      dfree(e->d_text);
      e->d_text = nullptr;
      e->d_text_cap = 0;
      int rc = dalloc(e, (void**)&e->d_text, len + 64);
      if (rc) return rc;
      e->d_text_cap = len;
    }
    readers = file_readers();
    chunk = file_chunk();
    shared = file_shared_stream();
    if (e->file_pin_bytes != chunk) {  // (re)size the pinned buffers
      for (int t = 0; t < MAX_FILE_READERS; t++)
        for (int k = 0; k < 2; k++)
          if (e->file_pin[t][k]) { (void)hipHostFree(e->file_pin[t][k]); e->file_pin[t][k] = nullptr; }
      e->file_pin_bytes = chunk;
    }
    for (int t = 0; t < readers; t++) {
      if (!e->file_stream[t]) HIPCHK(hipStreamCreateWithFlags(&e->file_stream[t], hipStreamNonBlocking));
      for (int k = 0; k < 2; k++) {
        if (!e->file_pin[t][k]) HIPCHK(hipHostMalloc((void**)&e->file_pin[t][k], chunk, hipHostMallocDefault));
        if (!e->file_ev[t][k]) HIPCHK(hipEventCreateWithFlags(&e->file_ev[t][k], hipEventDisableTiming));
      }
    }
    nchunks = (len + chunk - 1) / chunk;
    issued.assign(nchunks, 0);
    err.assign(readers, 0);
    msg.assign(readers, std::string());
    t0 = std::chrono::steady_clock::now();
    for (int t = 0; t < readers; t++) th.emplace_back([this, t] { reader(t); });
    return MOX_OK;
  }

  void abort_with(int t, int code, const char* m) {
    err[t] = code;
    msg[t] = m;
    std::lock_guard<std::mutex> g(mu);
    failed = true;
    cv.notify_all();
  }

  void reader(int t) {
    (void)hipSetDevice(e->device);
    hipStream_t cs = e->file_stream[shared ? 0 : t];
    int k = 0;
    bool used[2] = {false, false};
    for (size_t c = t; c < nchunks && !failed; c += readers, k ^= 1) {
      if (used[k] && hipEventSynchronize(e->file_ev[t][k]) != hipSuccess)  // buffer k's previous copy
        return abort_with(t, MOX_EHIP, "file copy failed");
      const size_t off = c * chunk, n = std::min(chunk, len - off);
      size_t got = 0;
      while (got < n) {
        const ssize_t r = pread(fd, e->file_pin[t][k] + got, n - got, (off_t)(off0 + off + got));
        if (r < 0 && errno == EINTR) continue;
        if (r <= 0) return abort_with(t, MOX_EIO, (std::string("read failed: ") + (r < 0 ? strerror(errno) : "short file")).c_str());
        got += (size_t)r;
      }
      // (another reader's copy may slip in between the copy and the record: the
      // event then completes a little later, which only delays the refill)
      if (hipMemcpyAsync(e->d_text + off, e->file_pin[t][k], n, hipMemcpyHostToDevice, cs) != hipSuccess ||
          hipEventRecord(e->file_ev[t][k], cs) != hipSuccess)
        return abort_with(t, MOX_EHIP, "hipMemcpyAsync failed");
      used[k] = true;
      std::lock_guard<std::mutex> g(mu);
      issued[c] = 1;
      while (prefix < nchunks && issued[prefix]) prefix++;
      cv.notify_all();
    }
    if (!shared && hipStreamSynchronize(cs) != hipSuccess) abort_with(t, MOX_EHIP, "file copy failed");
  }

  // true once the copies of bytes [0, bytes) are enqueued; false on a reader error
  bool wait_bytes(size_t bytes) {
    std::unique_lock<std::mutex> g(mu);
    cv.wait(g, [&] { return failed || prefix * chunk >= bytes || prefix == nchunks; });
    return !failed;
  }

  int finish() {
    for (auto& x : th) x.join();
    th.clear();
    if (shared) HIPCHK(hipStreamSynchronize(copy_stream()));
    for (int t = 0; t < readers; t++)
      if (err[t]) return fail(err[t], "%s", msg[t].c_str());
    e->stats.ms_h2d = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return MOX_OK;
  }
};

int stage_file_range(mox_engine* e, int fd, uint64_t off0, size_t len) {
  FileStager st(e, fd, off0, len);
  if (int rc = st.start()) return rc;
  return st.finish();
}

// mox_count_file on one engine with the map overlapped with the ingest: the
// file is read in chunks by the FileStager, and the map runs one launch per
// MAP_RANGE bytes as soon as that range and the next one (its look-ahead for
// tokens that cross the range end) have landed; the dictionary comes from a
// sample of the first range.  After the last range: the reduce tail of an
// ordinary pass over the whole file.  A token longer than the look-ahead or
// an overflow re-runs the pass on the now resident file (run_corpus), so the
// result is the ordinary pass's in every case.
constexpr size_t MAP_RANGE = 64ull << 20;
int run_file_overlapped(mox_engine* e, int fd, size_t len) {
  FileStager st(e, fd, 0, len);
  if (int rc = st.start()) return rc;
  if (e->dstream) HIPCHK(hipStreamSynchronize(e->dstream));
  e->have_result = false;
  const Corpus whole = make_corpus(e->d_text, len, 0, len, 1);
  Caps want = caps_max(initial_caps(len, e->n_cu), e->grow_hint);
  want.cold_cap = std::max<uint64_t>(want.cold_cap, e->next_cold_cap);
  if (int rc = ensure_caps(e, want)) return rc;
  e->grow_hint = Caps{};
  e->stats.retries = 0;
  if (!e->file_land) HIPCHK(hipEventCreateWithFlags(&e->file_land, hipEventDisableTiming));
  Work& w = e->w;
  hipStream_t s = e->stream;
  const Seq q = seq_of(e);
  // the engine stream waits until bytes [0, b) have landed
  auto land = [&](size_t b) -> int {
    if (!st.wait_bytes(b)) return MOX_EIO;  // the reader's error is reported by finish()
    HIPCHK(hipEventRecord(e->file_land, st.copy_stream()));
    HIPCHK(hipStreamWaitEvent(s, e->file_land, 0));
    return MOX_OK;
  };
  const size_t nr = (len + MAP_RANGE - 1) / MAP_RANGE;
  int rc = land(std::min(len, 2 * MAP_RANGE));
  if (!rc) {
    q.rec(0);
    const bool dict = !(e->flags & MOX_F_NO_DICT);
    hipLaunchKernelGGL(k_init, dim3(256), dim3(256), 0, s, w, 0ull, dict ? 1u : 0u);  // INIT_DICT
    if (dict) launch_dict(e, make_corpus(e->d_text, MAP_RANGE, 0, MAP_RANGE, 0), s, q);
    q.rec(1);
    for (size_t j = 0; j < nr && !rc; j++) {
      const size_t lo = j * MAP_RANGE, hi = std::min(len, lo + MAP_RANGE), ahead = std::min(len, hi + MAP_RANGE);
      if (j > 0) rc = land(ahead);
      if (rc) break;
      const Corpus cj = make_corpus(e->d_text, ahead, lo, hi, ahead == len);
      const uint64_t row0 = cj.own_lo & ~15ull;
      const uint64_t nrows = (cj.own_hi - row0 + PAY - 1) / PAY;
      hipLaunchKernelGGL(k_map, dim3(w.map_grid), dim3(MAP_THREADS), map_lds_bytes(), s, cj, w, nrows, j > 0 ? 1u : 0u);
    }
    if (!rc) {
      q.rec(2);
      hipLaunchKernelGGL(k_unicode, dim3(1024), dim3(256), 0, s, whole, w, e->tables);
      q.rec(3);
      launch_reduce_tail(e, whole, q);
    }
  }
  const int frc = st.finish();  // joins the readers: their error first
  if (frc) { (void)hipStreamSynchronize(s); return frc; }
  if (rc) { (void)hipStreamSynchronize(s); return fail(rc, "file ingest failed"); }
  const double h2d = e->stats.ms_h2d;
  if ((rc = finish_pass(e, q))) return rc;
  e->stats.ms_h2d = h2d;
  const Ctl& h = *e->h_ctl;
  if ((rc = check_failed(h))) return rc;
  if (h.err_utf8 != ~0ull) return fail(MOX_EUTF8, "stream did not contain valid UTF-8 (byte %llu)", h.err_utf8);
  if (h.halo_err != ~0ull || h.overflow) {  // a token past the look-ahead, or buffers too small: the ordinary pass
    if (h.overflow && !(h.overflow & OVF_REDUCE)) e->grow_hint = grow_for(e, h);
    rc = run_corpus(e, whole);
    e->stats.ms_h2d = h2d;
    return rc;
  }
  commit_result(e, whole, h);
  return MOX_OK;
}

}  // namespace mox_host

// ============================================================== C ABI
extern "C" {

const char* mox_last_error(void) { return g_err.c_str(); }
int mox_abi_version(void) { return MOX_ABI_VERSION; }

int mox_set_flags(mox_engine* e, uint32_t flags) {
  if (!e) return fail(MOX_EINVAL, "NULL engine");
  e->flags = flags;
  // an engine group: every member runs its shard's pass with the same flags
  // (timing modes, dictionary); the group's result flags live in member 0
  for (int i = 1; i < mox_group_size(e); i++) mox_group_member(e, i)->flags = flags;
  return MOX_OK;
}

int mox_engine_create(const mox_config* cfg, mox_engine** out) {
  if (!out) return fail(MOX_EINVAL, "out is NULL");
  *out = nullptr;
  const uint32_t n = cfg ? cfg->n_gpus : 0;
  if (n > MOX_MAX_GPUS) return fail(MOX_EINVAL, "n_gpus %u > %d", n, MOX_MAX_GPUS);
  if (cfg && cfg->n_devices && cfg->n_devices != n) return fail(MOX_EINVAL, "n_devices %u != n_gpus %u", cfg->n_devices, n);
  const int dev0 = cfg && cfg->n_devices ? cfg->devices[0] : (cfg ? cfg->device : -1);
  mox_engine* e = nullptr;
  if (int rc = engine_create_one(cfg, n > 1 && dev0 < 0 ? 0 : dev0, &e)) return rc;
  if (n > 1) {  // engine group: this engine is member 0 (mox_multi.hip)
    if (int rc = group_create(e, cfg)) {
      const std::string msg = g_err;
      mox_engine_destroy(e);
      g_err = msg;
      return rc;
    }
  }
  *out = e;
  return MOX_OK;
}

void mox_engine_destroy(mox_engine* e) {
  if (!e) return;
  if (e->grp) group_destroy(e);  // the other members and the communicators
  xplan_free(e);
  bsort_free(e);
  (void)hipSetDevice(e->device);
  (void)hipDeviceSynchronize();
  for (auto& a : e->aslot) {
    if (a.h_ctl) (void)hipHostFree(a.h_ctl);
    for (hipEvent_t ev : {a.ev_map0, a.ev_map1, a.ev_done}) if (ev) (void)hipEventDestroy(ev);
  }
  if (e->comm) ncclCommDestroy(e->comm);
  Work& w = e->w;
  for (auto& d : e->dsets)
    for (void* p : {(void*)d.cand, (void*)d.dict_hist, (void*)d.dict_list, (void*)d.dict_tag, (void*)d.dict_key, (void*)d.dict_tot}) dfree(p);
  void* ptrs[] = {w.ctl, w.cold_n, w.samp, w.spill_n, w.b_recs, (void*)e->tables.lower_src,
                  w.cold, w.spill, w.w, w.w_sorted, w.u, w.arena, w.ltab, w.lpos,
                  w.uk, w.uc, w.ui, w.t_counts, w.t_offs, w.t_bytes, e->d_text,
                  w.b_kk, w.red_order, w.u_base, w.sub_hist, w.sp_off, w.spw_off, w.udesc, w.big_units, w.mid_units, w.small_units, w.u_uniq, w.u_uniq_off,
                  w.u_bytes, w.u_bytes_off, w.b_bytes, w.split_k, w.split_w};
  for (void* p : ptrs) dfree(p);
  for (DevBuf* b : {&e->x_send_short, &e->x_send_blob, &e->x_recv_short, &e->x_recv_blob, &e->g_counts, &e->g_offs,
                    &e->g_bytes, &e->g_recv})
    dfree(b->p);
  for (DevBuf* b : {&e->hx_send, &e->hx_recv}) if (b->p) (void)hipHostFree(b->p);
  dfree(e->d_xcnt);
  dfree(e->d_xcur);
  dfree(e->d_xs);
  dfree(e->d_xr);
  dfree(e->d_xsp);
  if (e->h_xflag) (void)hipHostFree(e->h_xflag);
  if (e->ev_xs) (void)hipEventDestroy(e->ev_xs);
  if (e->h_xcnt) (void)hipHostFree(e->h_xcnt);
  if (e->h_ctl_x) (void)hipHostFree(e->h_ctl_x);
  if (e->h_ctl) (void)hipHostFree(e->h_ctl);
  if (e->h_ctl_init) (void)hipHostFree(e->h_ctl_init);
  for (auto& ev : e->ev) if (ev) (void)hipEventDestroy(ev);
  for (int t = 0; t < 16; t++) {
    if (e->file_stream[t]) (void)hipStreamDestroy(e->file_stream[t]);
    for (int k = 0; k < 2; k++) {
      if (e->file_ev[t][k]) (void)hipEventDestroy(e->file_ev[t][k]);
      if (e->file_pin[t][k]) (void)hipHostFree(e->file_pin[t][k]);
    }
  }
  if (e->file_land) (void)hipEventDestroy(e->file_land);
  if (e->stream) (void)hipStreamDestroy(e->stream);
  if (e->dstream) (void)hipStreamDestroy(e->dstream);
  if (e->ev_dready) (void)hipEventDestroy(e->ev_dready);
  if (e->ev_mapped) (void)hipEventDestroy(e->ev_mapped);
  delete e;
}

int mox_run_range_async(mox_engine* e, const void* d_buf, size_t buf_len, size_t own_begin, size_t own_end,
                        int at_corpus_end) {
  if (!e) return fail(MOX_EINVAL, "engine is NULL");
  if (e->grp) return fail(MOX_EINVAL, "engine group: one shard per GPU (mox_run_shards)");
  if (!d_buf && buf_len) return fail(MOX_EINVAL, "buffer is NULL");
  if (own_begin > own_end || own_end > buf_len) return fail(MOX_EINVAL, "bad own range [%zu, %zu) of %zu", own_begin, own_end, buf_len);
  if (own_begin > 0 && own_begin < 4) return fail(MOX_EINVAL, "own_begin must be 0 (corpus start) or >= 4 (left context)");
  HIPCHK(hipSetDevice(e->device));
  const Corpus c = make_corpus(buf_len ? d_buf : (const void*)e->w.ctl, buf_len, own_begin, own_end, at_corpus_end);
  const int k = e->anext;
  auto& a = e->aslot[k];
  if (a.pending) {  // two passes already queued: complete the older one first
    int rc = complete_async(e, k);
    if (rc) return rc;
  }
  if (!a.h_ctl) {
    HIPCHK(hipHostMalloc((void**)&a.h_ctl, sizeof(Ctl), hipHostMallocDefault));
    HIPCHK(hipEventCreate(&a.ev_map0));
    HIPCHK(hipEventCreate(&a.ev_map1));
    HIPCHK(hipEventCreateWithFlags(&a.ev_done, hipEventDisableTiming));
  }
  Caps want = caps_max(initial_caps(c.own_hi - c.own_lo, e->n_cu), e->grow_hint);
  want.cold_cap = std::max<uint64_t>(want.cold_cap, e->next_cold_cap);
  if (!(e->w.cold && caps_cover(caps_of(e->w), want))) {
    // a regrow frees the buffers a pending pass wrote its table into: complete
    // (check, commit) pending passes first
    if (int rc = drain_async(e)) return rc;
  }
  int rc = ensure_caps(e, want);
  if (rc) return rc;
  e->grow_hint = Caps{};
  e->have_result = false;
  Seq q = seq_of(e);
  q.map_ev[0] = a.ev_map0;
  q.map_ev[1] = a.ev_map1;
  enqueue_pass(e, c, q, /*side=*/true);
  HIPCHK(hipGetLastError());
  static_assert(sizeof(Ctl) / 8 <= 256, "k_ctl_out: one workgroup");
  hipLaunchKernelGGL(k_ctl_out, dim3(1), dim3(256), 0, e->stream, (const Ctl*)e->w.ctl, a.h_ctl);
  HIPCHK(hipEventRecord(a.ev_done, e->stream));
  a.pending = true;
  a.c = c;
  e->anext = k ^ 1;
  // the previous pass, if any, completes while this one is already queued
  return complete_async(e, k ^ 1);
}

int mox_run_wait(mox_engine* e) {
  if (!e) return fail(MOX_EINVAL, "engine is NULL");
  HIPCHK(hipSetDevice(e->device));
  return drain_async(e);
}

int mox_run_range(mox_engine* e, const void* d_buf, size_t buf_len, size_t own_begin, size_t own_end, int at_corpus_end) {
  if (!e) return fail(MOX_EINVAL, "engine is NULL");
  if (e->grp) return fail(MOX_EINVAL, "engine group: one shard per GPU (mox_run_shards)");
  if (int rc = drain_async(e)) return rc;
  if (!d_buf && buf_len) return fail(MOX_EINVAL, "buffer is NULL");
  if (own_begin > own_end || own_end > buf_len) return fail(MOX_EINVAL, "bad own range [%zu, %zu) of %zu", own_begin, own_end, buf_len);
  if (own_begin > 0 && own_begin < 4) return fail(MOX_EINVAL, "own_begin must be 0 (corpus start) or >= 4 (left context)");
  HIPCHK(hipSetDevice(e->device));
  // an empty corpus has no tokens (reference: empty file -> empty map); any
  // valid device address serves as its base
  Corpus c = make_corpus(buf_len ? d_buf : (const void*)e->w.ctl, buf_len, own_begin, own_end, at_corpus_end);
  return run_corpus(e, c);
}

int mox_run_device(mox_engine* e, const void* d_text, size_t len) { return mox_run_range(e, d_text, len, 0, len, 1); }

int mox_fetch_table(mox_engine* e, mox_table** out) {
  if (!e || !out) return fail(MOX_EINVAL, "NULL argument");
  *out = nullptr;
  if (int rc = drain_async(e)) return rc;
  if (!e->have_result) return fail(MOX_ESTATE, "no result: run first");
  HIPCHK(hipSetDevice(e->device));
  // MOX_F_SORT_BYTES: bytewise order on the GPU (mox_bsort.hip) before the copy;
  // a table too big for the sort's device scratch is sorted on the host below
  bool host_sort = false;
  if ((e->flags & MOX_F_SORT_BYTES) && !e->res.sorted) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = bsort_table(e);
    if (rc == MOX_ENOMEM) host_sort = true;
    else if (rc) return rc;
    e->stats.ms_sort = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  const bool timing = (e->flags & MOX_F_TIMING) != 0;
  if (timing) HIPCHK(hipEventRecord(e->ev[6], e->stream));
  const mox_engine::Res& r = e->res;
  uint64_t n = r.n, nb = r.nb;
  size_t bytes = sizeof(mox_table) + (n + 1) * 8 * 2 + nb + 16;
  uint8_t* mem = (uint8_t*)malloc(bytes);
  if (!mem) return fail(MOX_ENOMEM, "host allocation of %zu bytes failed", bytes);
  mox_table* t = (mox_table*)mem;
  uint64_t* counts = (uint64_t*)(mem + sizeof(mox_table));
  uint64_t* offs = counts + n + 1;
  uint8_t* wb = (uint8_t*)(offs + n + 1);
  t->n = n;
  t->tokens = r.tokens;
  t->counts = counts;
  t->offs = offs;
  t->bytes = wb;
  if (n) {
    HIPCHK(hipMemcpyAsync(counts, r.counts, n * 8, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(offs, r.offs, (n + 1) * 8, hipMemcpyDeviceToHost, e->stream));
    if (nb) HIPCHK(hipMemcpyAsync(wb, r.bytes, nb, hipMemcpyDeviceToHost, e->stream));
  } else {
    offs[0] = 0;
  }
  if (timing) HIPCHK(hipEventRecord(e->ev[7], e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  if (timing) e->stats.ms_d2h = ev_ms(e, 6, 7);
  if (host_sort) {
    if (int rc = mox_table_sort_bytes(t)) {
      free(mem);
      return rc;
    }
  }
  *out = t;
  return MOX_OK;
}

int mox_sort_result(mox_engine* e) {
  if (!e) return fail(MOX_EINVAL, "NULL argument");
  if (int rc = drain_async(e)) return rc;
  if (!e->have_result) return fail(MOX_ESTATE, "no result: run first");
  if (e->res.sorted) return MOX_OK;
  const auto t0 = std::chrono::steady_clock::now();
  const int rc = bsort_table(e);
  e->stats.ms_sort = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return rc;
}

void mox_table_free(mox_table* t) { free(t); }

int mox_table_sort_bytes(mox_table* t) {
  if (!t) return fail(MOX_EINVAL, "NULL argument");
  try {
    if (mox_host::sort_table_bytes(t->n, const_cast<uint64_t*>(t->counts), const_cast<uint64_t*>(t->offs),
                                   const_cast<uint8_t*>(t->bytes)) != 0)
      return fail(MOX_ENOMEM, "host allocation failed while sorting the table");
  } catch (const std::exception& ex) {
    return fail(MOX_ENOMEM, "sorting the table failed: %s", ex.what());
  }
  return MOX_OK;
}

int mox_get_stats(const mox_engine* e, mox_stats* out) {
  if (!e || !out) return fail(MOX_EINVAL, "NULL argument");
  *out = e->stats;
  return MOX_OK;
}

int mox_count(mox_engine* e, const uint8_t* text, size_t len, mox_table** out) {
  if (!e || !out || (!text && len)) return fail(MOX_EINVAL, "NULL argument");
  *out = nullptr;
  HIPCHK(hipSetDevice(e->device));
  if (int rc = drain_async(e)) return rc;
  if (e->grp) {  // engine group: byte ranges at whitespace, one per GPU (mox_multi.hip)
    if (int rc = group_count_host(e, text, len)) return rc;
    return mox_fetch_table(e, out);
  }
  int rc = stage_host_range(e, text, len);
  if (rc) return rc;
  if ((rc = mox_run_range(e, len ? (const void*)e->d_text : nullptr, len, 0, len, 1))) return rc;
  return mox_fetch_table(e, out);
}

int mox_count_file(mox_engine* e, const char* path, mox_table** out) {
  if (!e || !path || !out) return fail(MOX_EINVAL, "NULL argument");
  *out = nullptr;
  HIPCHK(hipSetDevice(e->device));
  if (int rc = drain_async(e)) return rc;
  if (e->grp) {  // engine group: every GPU reads its own byte range of the file
    if (int rc = group_count_file(e, path)) return rc;
    return mox_fetch_table(e, out);
  }
  int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(MOX_EIO, "cannot open %s: %s", path, strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) { close(fd); return fail(MOX_EIO, "cannot stat %s: %s", path, strerror(errno)); }
  const size_t len = (size_t)st.st_size;
  if (len > 2 * MAP_RANGE && file_shared_stream()) {  // big file: the map overlaps the ingest
    const int rc = run_file_overlapped(e, fd, len);
    close(fd);
    if (rc) return rc;
    return mox_fetch_table(e, out);
  }
  int rc = stage_file_range(e, fd, 0, len);
  close(fd);
  if (rc) return rc;
  const double h2d = e->stats.ms_h2d;
  if ((rc = mox_run_range(e, len ? (const void*)e->d_text : nullptr, len, 0, len, 1))) return rc;
  e->stats.ms_h2d = h2d;  // file read + copy wall time (PCIe-inclusive ingest)
  return mox_fetch_table(e, out);
}

int mox_device_alloc(mox_engine* e, size_t bytes, void** d_ptr) {
  if (!e || !d_ptr) return fail(MOX_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(e->device));
  return dalloc(e, d_ptr, bytes);
}
int mox_device_free(mox_engine* e, void* d_ptr) {
  if (!e) return fail(MOX_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(e->device));
  if (d_ptr) HIPCHK(hipFree(d_ptr));
  return MOX_OK;
}
int mox_memcpy_h2d(mox_engine* e, void* d_dst, const void* h_src, size_t bytes) {
  if (!e || (!d_dst && bytes) || (!h_src && bytes)) return fail(MOX_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(e->device));
  if (bytes) HIPCHK(hipMemcpyAsync(d_dst, h_src, bytes, hipMemcpyHostToDevice, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return MOX_OK;
}
int mox_memcpy_d2h(mox_engine* e, void* h_dst, const void* d_src, size_t bytes) {
  if (!e || (!d_src && bytes) || (!h_dst && bytes)) return fail(MOX_EINVAL, "NULL argument");
  HIPCHK(hipSetDevice(e->device));
  if (bytes) HIPCHK(hipMemcpyAsync(h_dst, d_src, bytes, hipMemcpyDeviceToHost, e->stream));
  HIPCHK(hipStreamSynchronize(e->stream));
  return MOX_OK;
}
int mox_synchronize(mox_engine* e) {
  if (!e) return fail(MOX_EINVAL, "NULL argument");
  if (int rc = drain_async(e)) return rc;  // queued passes complete (and are checked) first
  HIPCHK(hipStreamSynchronize(e->stream));
  return MOX_OK;
}

// ---- output layer (reference L5) ----
int mox_write_final_result(const mox_table* t, const char* path) {
  if (!t || !path) return fail(MOX_EINVAL, "NULL argument");
  FILE* f = fopen(path, "wb");
  if (!f) return fail(MOX_EIO, "cannot open %s: %s", path, strerror(errno));
  std::vector<char> buf;
  buf.reserve(1 << 20);
  char num[32];
  for (uint64_t i = 0; i < t->n; i++) {
    buf.insert(buf.end(), t->bytes + t->offs[i], t->bytes + t->offs[i + 1]);
    int k = snprintf(num, sizeof num, " %llu\n", (unsigned long long)t->counts[i]);
    buf.insert(buf.end(), num, num + k);
    if (buf.size() > (1u << 20)) {
      if (fwrite(buf.data(), 1, buf.size(), f) != buf.size()) { fclose(f); return fail(MOX_EIO, "write failed"); }
      buf.clear();
    }
  }
  if (!buf.empty() && fwrite(buf.data(), 1, buf.size(), f) != buf.size()) { fclose(f); return fail(MOX_EIO, "write failed"); }
  if (fclose(f) != 0) return fail(MOX_EIO, "close failed");
  return MOX_OK;
}

int mox_print_top_words(const mox_table* t, size_t n) {
  if (!t) return fail(MOX_EINVAL, "NULL argument");
  std::vector<uint64_t> idx(t->n);
  for (uint64_t i = 0; i < t->n; i++) idx[i] = i;
  size_t k = std::min<size_t>(n, t->n);
  std::partial_sort(idx.begin(), idx.begin() + k, idx.end(), [&](uint64_t a, uint64_t b) {
    if (t->counts[a] != t->counts[b]) return t->counts[a] > t->counts[b];
    return a < b;
  });
  printf("Top %zu words:\n", n);
  for (size_t i = 0; i < k; i++) {
    uint64_t j = idx[i];
    printf("%.*s: %llu\n", (int)(t->offs[j + 1] - t->offs[j]), (const char*)t->bytes + t->offs[j],
           (unsigned long long)t->counts[j]);
  }
  return MOX_OK;
}

}  // extern "C"
