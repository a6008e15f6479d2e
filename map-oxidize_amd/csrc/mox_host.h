// Host side of libmox.so: the engine object and the helpers shared by the
// pass driver (mox_engine.hip), the multi-GPU exchange / gather / engine group
// (mox_multi.hip) and the device bytewise table sort (mox_bsort.hip).  Internal:
// the public interface is include/mox.h.
#pragma once
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <condition_variable>
#include <chrono>
#include <cstdarg>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/mox.h"
#include "mox_internal.h"
#include "mox_table.h"

using namespace mox;

extern "C" {
__global__ void k_map(Corpus c, Work w, uint64_t nrows, uint32_t resume);
__global__ void k_init(Work w, unsigned long long w_n, uint32_t flags);
__global__ void k_ctl_out(const Ctl* src, Ctl* dst);
__global__ void k_sample(Corpus c, Work w, uint32_t npieces);
__global__ void k_dict_hist(Work w);
__global__ void k_dict_pick(Work w, uint32_t max_words);
__global__ void k_dict_build(Work w, uint32_t max_words);
__global__ void k_dict_zero(Work w);
__global__ void k_unicode(Corpus c, Work w, Tables T);
__global__ void k_hist(Work w);
__global__ void k_scatter(Work w);
__global__ void k_reduce(Work w);
__global__ void k_split_count(Work w);
__global__ void k_unit_scan(Work w);
__global__ void k_split_scatter(Work w);
__global__ void k_unit_uniq_scan(Work w);
__global__ void k_final_scan(Work w);
__global__ void k_reduce_small(Work w);
__global__ void k_reduce_sort1(Work w);
__global__ void k_reduce_sort2(Work w);
__global__ void k_mat(Work w, Corpus c);
__global__ void k_xcount(Work w, uint32_t P, XCnt* xcnt);
__global__ void k_xpack_short(Work w, WRec* out);
__global__ void k_xpack_long(Work w, XDir dir, unsigned long long* cur, uint8_t* blob);
__global__ void k_xsample(Work w, uint64_t* out);
__global__ void k_xsplit(const uint64_t* blocks, uint32_t P, uint64_t* sp, uint32_t* flag);
__global__ void k_xcount_r(Work w, XSplit x, XCnt* xcnt);
__global__ void k_xpack_r(Work w, XSplit x, XDir dir, unsigned long long* cur, WRec* out, uint8_t* blob);
__global__ void k_xingest(Work w, XDir dir, uint64_t n_short);
__global__ void k_gather_offs(const uint8_t* recv, GDir d, uint64_t* out);
}

namespace mox_host {
// Buffer-growth reruns of one pass: every overflow kind grows its buffers in
// one step, but an attempt that overflowed early (cold regions, the split
// layout) does not reach the later checks (table, bytes), so the kinds can be
// met one attempt after another
constexpr int GROW_RETRIES = 8;


// thread-local last error (mox_last_error) and the status-returning setter
extern thread_local std::string g_err;
int fail(int code, const char* fmt, ...) __attribute__((format(printf, 2, 3)));

#define HIPCHK(expr)                                                                             \
  do {                                                                                           \
    hipError_t e_ = (expr);                                                                      \
    if (e_ != hipSuccess) return fail(MOX_EHIP, "%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
  } while (0)

#define RCCLCHK(expr)                                                                            \
  do {                                                                                           \
    ncclResult_t r_ = (expr);                                                                    \
    if (r_ != ncclSuccess) return fail(MOX_ERCCL, "%s failed: %s", #expr, ncclGetErrorString(r_)); \
  } while (0)

inline uint64_t next_pow2(uint64_t x) {
  uint64_t p = 1;
  while (p < x) p <<= 1;
  return p;
}

struct DevBuf {
  void* p = nullptr;
  size_t cap = 0;
};
// Capacities of the size-dependent pass buffers.
struct Caps {
  uint64_t cold_cap, spill_cap, w_cap, u_cap, arena_cap, long_cap, table_cap, bytes_cap, split_k_cap, split_w_cap;
};
struct XPlan;  // mox_multi.hip
struct Group;  // mox_multi.hip

}  // namespace mox_host

using namespace mox_host;

struct mox_engine {
  int device = 0;
  hipStream_t stream = nullptr;
  // async passes: pass k + 1's dictionary is built on dstream while pass k's
  // reduce tail runs on stream (ev_dready: the next dictionary is built).  The
  // dictionary buffers are double-buffered (dsets): a side build writes the set
  // the previous pass did not use, and the pass before that one has completed
  // on the host by then (mox_run_range_async completes pass k - 1 before it
  // returns), so the side stream waits for nothing.
  hipStream_t dstream = nullptr;
  hipEvent_t ev_dready = nullptr;
  // MOX_SIDE_AFTER_MAP=1 (mox_engine.hip): recorded right after an async
  // pass's k_map, and the next pass's side build waits for it, so that the
  // build runs beside the reduce tail rather than beside k_map (where the
  // trace shows k_sample stretching k_map's launches by 10-120 us).  Measured
  // 1.1 % slower end to end (the tail pays more than k_map saves), so off by
  // default (profiles/r05/c2_side_dict_overlap.txt).
  hipEvent_t ev_mapped = nullptr;
  bool mapped_pending = false;  // ev_mapped recorded by a pass whose successor has not waited on it yet
  struct DictSet {
    WRec* cand = nullptr;
    uint32_t* dict_hist = nullptr;
    WRec* dict_list = nullptr;
    uint32_t* dict_tag = nullptr;
    uint4* dict_key = nullptr;
    unsigned long long* dict_tot = nullptr;
  } dsets[2];
  int dcur = 0;  // the set the last enqueued pass used (it is in e->w)
  uint32_t flags = 0, dict_words = DICT_MAX_WORDS, sample_pieces = 192;
  int n_cu = 256;
  bool sync_each = false;
  bool verbose = false;         // MOX_VERBOSE: one line per pass attempt on stderr
  int test_fail_alloc = 0;     // MOX_TEST_FAIL_ALLOC=k: the k-th sized allocation fails once (tests)
  uint64_t next_cold_cap = 0;  // region capacity learnt from spills of an earlier run
  Caps grow_hint{};            // capacities an overflowed, superseded async pass asked for (next run)
  Work w{};
  Tables tables{};
  Ctl* h_ctl = nullptr;       // pinned
  Ctl* h_ctl_init = nullptr;  // pinned
  // engine-owned corpus staging for host inputs
  uint8_t* d_text = nullptr;
  size_t d_text_cap = 0;
  hipStream_t file_stream[16]{};  // mox_count_file readers (up to MAX_FILE_READERS); [0] = the shared copy stream
  hipEvent_t file_ev[16][2]{};    // copy of reader t's buffer k done (shared copy stream)
  hipEvent_t file_land = nullptr; // overlapped file pass: copies of a byte prefix done (shared copy stream)
  uint8_t* file_pin[16][2]{};
  size_t file_pin_bytes = 0;      // size of each pinned reader buffer
  // last run
  bool have_result = false;
  // where the result table lives (the pass's t_* buffers, or the gather buffers)
  struct Res {
    const uint64_t* counts = nullptr;
    const uint64_t* offs = nullptr;
    const uint8_t* bytes = nullptr;
    uint64_t n = 0, nb = 0, tokens = 0;
    bool pass = false;       // true: the t_* buffers of the last pass (an exchange can start from it)
    bool exchanged = false;  // true: the final table of an exchange (this rank's words are final: gatherable)
    bool sorted = false;     // true: in bytewise order (bsort_table)
  } res;
  DevBuf g_counts, g_offs, g_bytes, g_recv;  // mox_gather (root)
  DevBuf s_counts, s_offs, s_bytes, s_tmp;    // device bytewise sort (mox_bsort.hip): output + scratch
  unsigned long long* h_bsort = nullptr;      // pinned: the sort's digit histograms + totals
  Corpus last_corpus{};
  mox_stats stats{};
  hipEvent_t ev[12]{};
  // mox_run_range_async: two pass slots (the newest pass is enqueued before the
  // previous one is completed, so the GPU runs them back to back)
  struct AsyncSlot {
    bool pending = false;
    Corpus c{};
    Ctl* h_ctl = nullptr;                  // pinned copy of this pass's control block
    hipEvent_t ev_map0 = nullptr, ev_map1 = nullptr, ev_done = nullptr;
  } aslot[2];
  int anext = 0;
  // multi-GPU, one process per GPU (mox_comm_init)
  ncclComm_t comm = nullptr;
  int nranks = 1, rank = 0;
  XCnt* d_xcnt = nullptr;                 // [0, MAX_RANKS) sent, [MAX_RANKS, 2 MAX_RANKS) received
  XCnt* h_xcnt = nullptr;                 // pinned mirror
  unsigned long long* d_xcur = nullptr;   // 3 MAX_RANKS pack cursors
  uint64_t* d_xs = nullptr;               // sorted exchange: MAX_RANKS x XS_BLOCK sample blocks sent (one copy per peer)
  uint64_t* d_xr = nullptr;               // ... and received
  uint64_t* d_xsp = nullptr;              // MAX_RANKS splitters (k_xsplit), then the skew flag word
  uint32_t* h_xflag = nullptr;            // pinned copy of the skew flag
  hipEvent_t ev_xs = nullptr;             // engine group, copy transport: this member's sample block is written
  DevBuf x_send_short, x_send_blob, x_recv_short, x_recv_blob;  // device
  DevBuf hx_send, hx_recv;                // pinned host staging (host transport)
  Ctl* h_ctl_x = nullptr;                 // pinned control block of an exchange pass
  XPlan* xp = nullptr;                    // layout of the exchange in progress (mox_multi.hip)
  // engine group (mox_config.n_gpus > 1): this engine is member 0 and drives
  // the others from one host thread (mox_multi.hip)
  Group* grp = nullptr;
};

namespace mox_host {
// ---- mox_engine.hip
int dalloc(mox_engine* e, void** p, size_t bytes);
void dfree(void* p);
Caps caps_of(const Work& w);
Caps initial_caps(uint64_t n, int map_grid);
Caps caps_max(const Caps& a, const Caps& b);
int ensure_caps(mox_engine* e, const Caps& need);
Caps grow_for(mox_engine* e, const Ctl& h);
int check_failed(const Ctl& h);
void set_result(mox_engine* e, const Ctl& h);
int drain_async(mox_engine* e);
int run_corpus(mox_engine* e, const Corpus& c);
Corpus make_corpus(const void* d_buf, size_t buf_len, size_t own_begin, size_t own_end, int at_end);
// Launch sequencing helpers: HIP-event timestamps (MOX_F_TIMING) and, with
// MOX_SYNC_EACH=1, a synchronisation + name after every launch (hang / fault
// triage).
struct Seq {
  mox_engine* e;
  hipStream_t s;
  bool timing, sync_each, map_only;
  hipEvent_t map_ev[2] = {nullptr, nullptr};  // async passes: their own map events
  void rec(int i) const;
  void step(const char* name) const;
};
Seq seq_of(mox_engine* e);
void launch_reduce_tail(mox_engine* e, const Corpus& c, const Seq& q);
int finish_pass(mox_engine* e, const Seq& q);
int engine_create_one(const mox_config* cfg, int device, mox_engine** out);
int stage_host_range(mox_engine* e, const uint8_t* text, size_t len);
int stage_file_range(mox_engine* e, int fd, uint64_t off, size_t len);
// ---- mox_multi.hip
int grow_dev(DevBuf& b, size_t bytes);
int grow_pinned(DevBuf& b, size_t bytes);
void group_destroy(mox_engine* e);
int group_create(mox_engine* e, const mox_config* cfg);
int group_count_host(mox_engine* e, const uint8_t* text, size_t len);
int group_count_file(mox_engine* e, const char* path);
void xplan_free(mox_engine* e);
// ---- mox_bsort.hip
int bsort_table(mox_engine* e);  // the result table in bytewise order, on the device
void bsort_free(mox_engine* e);
}  // namespace mox_host
