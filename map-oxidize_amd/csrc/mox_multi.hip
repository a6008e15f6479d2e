// Multi-GPU side of libmox.so: the exchange of the ranks' partial
// tables, the gather of the final tables, and the engine group that runs
// both for several GPUs from one process and one host thread.
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstring>
#include <thread>

#include "mox_host.h"

namespace mox_host {

// ============================================================== multi-GPU exchange
//   After a local pass every rank holds a dense table of its
// byte range.  Each table row goes to the owner of its hash (short words:
// partition ranges, already contiguous per owner in the dense order; long
// words: FNV hash ranges, packed per owner).  The exchange is three
// all-to-alls (per-peer counts, short records, long blobs) over a transport,
// then one reduce-only pass over the received partials produces this rank's
// final table.  Ranks own disjoint word sets.

int grow_dev(DevBuf& b, size_t bytes) {
  if (b.cap >= bytes && b.p) return MOX_OK;
  dfree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
  hipError_t err = hipMalloc(&b.p, want);
  if (err != hipSuccess) {
    b.p = nullptr;
    (void)hipGetLastError();  // the failed allocation's error is not a later launch's (callers may fall back)
    return fail(MOX_ENOMEM, "hipMalloc(%zu) failed: %s", want, hipGetErrorString(err));
  }
  b.cap = want;
  return MOX_OK;
}
int grow_pinned(DevBuf& b, size_t bytes) {
  if (b.cap >= bytes && b.p) return MOX_OK;
  if (b.p) (void)hipHostFree(b.p);
  b.p = nullptr;
  b.cap = 0;
  size_t want = std::max<size_t>(bytes + bytes / 4, 4096);
  hipError_t err = hipHostMalloc(&b.p, want, hipHostMallocDefault);
  if (err != hipSuccess) return fail(MOX_ENOMEM, "hipHostMalloc(%zu) failed: %s", want, hipGetErrorString(err));
  b.cap = want;
  return MOX_OK;
}

// Moves per-peer byte ranges between ranks.  send/recv are device buffers;
// off/len are per-peer byte offsets and sizes (len identical on both sides of
// every pair by construction).
struct Transport {
  virtual ~Transport() = default;
  // per-peer count rows: d_send[d] (device, just written by k_xcount) -> peer
  // d; on return h_send holds this rank's rows and h_recv[s] peer s's rows.
  virtual int counts(const XCnt* d_send, XCnt* d_recv, XCnt* h_send, XCnt* h_recv) = 0;
  virtual int alltoallv(const uint8_t* send, const uint64_t* soff, const uint64_t* slen, uint8_t* recv, const uint64_t* roff,
                        const uint64_t* rlen) = 0;
  // two independent all-to-alls (short records, long-word blobs); a transport
  // may move both in one round
  virtual int alltoallv_pair(const uint8_t* send_a, const uint64_t* soff_a, const uint64_t* slen_a, uint8_t* recv_a,
                             const uint64_t* roff_a, const uint64_t* rlen_a, const uint8_t* send_b, const uint64_t* soff_b,
                             const uint64_t* slen_b, uint8_t* recv_b, const uint64_t* roff_b, const uint64_t* rlen_b) {
    int rc = alltoallv(send_a, soff_a, slen_a, recv_a, roff_a, rlen_a);
    return rc ? rc : alltoallv(send_b, soff_b, slen_b, recv_b, roff_b, rlen_b);
  }
};

struct RcclTransport : Transport {
  mox_engine* e;
  explicit RcclTransport(mox_engine* e_) : e(e_) {}
  int counts(const XCnt* d_send, XCnt* d_recv, XCnt* h_send, XCnt* h_recv) override {
    // device to device right after k_xcount: one host synchronisation for both rows
    const int P = e->nranks;
    RCCLCHK(ncclGroupStart());
    for (int p = 0; p < P; p++) {
      RCCLCHK(ncclSend(d_send + p, sizeof(XCnt), ncclUint8, p, e->comm, e->stream));
      RCCLCHK(ncclRecv(d_recv + p, sizeof(XCnt), ncclUint8, p, e->comm, e->stream));
    }
    RCCLCHK(ncclGroupEnd());
    HIPCHK(hipMemcpyAsync(h_send, d_send, P * sizeof(XCnt), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipMemcpyAsync(h_recv, d_recv, P * sizeof(XCnt), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    return MOX_OK;
  }
  int alltoallv(const uint8_t* send, const uint64_t* soff, const uint64_t* slen, uint8_t* recv, const uint64_t* roff,
                const uint64_t* rlen) override {
    const int P = e->nranks, me = e->rank;
    if (slen[me]) HIPCHK(hipMemcpyAsync(recv + roff[me], send + soff[me], slen[me], hipMemcpyDeviceToDevice, e->stream));
    RCCLCHK(ncclGroupStart());
    for (int p = 0; p < P; p++) {
      if (p == me) continue;
      if (slen[p]) RCCLCHK(ncclSend(send + soff[p], slen[p], ncclUint8, p, e->comm, e->stream));
      if (rlen[p]) RCCLCHK(ncclRecv(recv + roff[p], rlen[p], ncclUint8, p, e->comm, e->stream));
    }
    RCCLCHK(ncclGroupEnd());
    return MOX_OK;
  }
  // both payloads inside ONE ncclGroupStart/End: one RCCL launch and one round
  // of peer handshakes per exchange instead of two
  int alltoallv_pair(const uint8_t* send_a, const uint64_t* soff_a, const uint64_t* slen_a, uint8_t* recv_a,
                     const uint64_t* roff_a, const uint64_t* rlen_a, const uint8_t* send_b, const uint64_t* soff_b,
                     const uint64_t* slen_b, uint8_t* recv_b, const uint64_t* roff_b, const uint64_t* rlen_b) override {
    const int P = e->nranks, me = e->rank;
    if (slen_a[me]) HIPCHK(hipMemcpyAsync(recv_a + roff_a[me], send_a + soff_a[me], slen_a[me], hipMemcpyDeviceToDevice, e->stream));
    if (slen_b[me]) HIPCHK(hipMemcpyAsync(recv_b + roff_b[me], send_b + soff_b[me], slen_b[me], hipMemcpyDeviceToDevice, e->stream));
    if (P == 1) return MOX_OK;
    RCCLCHK(ncclGroupStart());
    for (int p = 0; p < P; p++) {
      if (p == me) continue;
      if (slen_a[p]) RCCLCHK(ncclSend(send_a + soff_a[p], slen_a[p], ncclUint8, p, e->comm, e->stream));
      if (rlen_a[p]) RCCLCHK(ncclRecv(recv_a + roff_a[p], rlen_a[p], ncclUint8, p, e->comm, e->stream));
      if (slen_b[p]) RCCLCHK(ncclSend(send_b + soff_b[p], slen_b[p], ncclUint8, p, e->comm, e->stream));
      if (rlen_b[p]) RCCLCHK(ncclRecv(recv_b + roff_b[p], rlen_b[p], ncclUint8, p, e->comm, e->stream));
    }
    RCCLCHK(ncclGroupEnd());
    return MOX_OK;
  }
};

// Host-staged transport: device -> pinned host, caller's all-to-all callback
// (e.g. torch.distributed over gloo), pinned host -> device.  Used where RCCL
// cannot run (several ranks sharing one GPU in tests).
struct HostTransport : Transport {
  mox_engine* e;
  int P;
  mox_alltoallv_fn fn;
  void* user;
  HostTransport(mox_engine* e_, int P_, mox_alltoallv_fn f, void* u) : e(e_), P(P_), fn(f), user(u) {}
  int counts(const XCnt* d_send, XCnt*, XCnt* h_send, XCnt* h_recv) override {
    HIPCHK(hipMemcpyAsync(h_send, d_send, P * sizeof(XCnt), hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    uint64_t len[MAX_RANKS];
    for (int p = 0; p < P; p++) len[p] = sizeof(XCnt);
    if (fn(user, h_send, len, h_recv, len) != 0) return fail(MOX_EIO, "host all-to-all callback failed (counts)");
    return MOX_OK;
  }
  int alltoallv(const uint8_t* send, const uint64_t* soff, const uint64_t* slen, uint8_t* recv, const uint64_t* roff,
                const uint64_t* rlen) override {
    const uint64_t stot = soff[P - 1] + slen[P - 1], rtot = roff[P - 1] + rlen[P - 1];
    int rc;
    // a previous call's H2D from hx_recv may still be in flight on the stream:
    // drain it before a regrow frees the pinned buffer under it
    if (e->hx_send.cap < stot + 8 || e->hx_recv.cap < rtot + 8) HIPCHK(hipStreamSynchronize(e->stream));
    if ((rc = grow_pinned(e->hx_send, stot + 8)) || (rc = grow_pinned(e->hx_recv, rtot + 8))) return rc;
    if (stot) HIPCHK(hipMemcpyAsync(e->hx_send.p, send, stot, hipMemcpyDeviceToHost, e->stream));
    HIPCHK(hipStreamSynchronize(e->stream));
    if (fn(user, e->hx_send.p, slen, e->hx_recv.p, rlen) != 0) return fail(MOX_EIO, "host all-to-all callback failed");
    if (rtot) HIPCHK(hipMemcpyAsync(recv, e->hx_recv.p, rtot, hipMemcpyHostToDevice, e->stream));
    return MOX_OK;
  }
};

// One attempt of the reduce-only pass over the received partials.
int exchange_pass_once(mox_engine* e, uint64_t r_short, uint64_t blob_bytes, const XDir& rdir) {
  Work& w = e->w;
  hipStream_t s = e->stream;
  const Seq q = seq_of(e);
  q.rec(0);
  // control block (w_n = received records), counters, long table, no map regions
  hipLaunchKernelGGL(k_init, dim3(256), dim3(256), 0, s, w, (unsigned long long)r_short, 2u);
  if (r_short) HIPCHK(hipMemcpyAsync(w.w, e->x_recv_short.p, r_short * sizeof(WRec), hipMemcpyDeviceToDevice, s));
  if (blob_bytes) HIPCHK(hipMemcpyAsync(w.arena, e->x_recv_blob.p, blob_bytes, hipMemcpyDeviceToDevice, s));
  q.rec(1);
  q.rec(2);
  hipLaunchKernelGGL(k_xingest, dim3(1024), dim3(256), 0, s, w, rdir, r_short);
  q.step("k_xingest");
  q.rec(3);
  Corpus none{};
  none.base = (const uint8_t*)w.ctl;  // long refs are all arena refs in this pass
  launch_reduce_tail(e, none, q);
  return finish_pass(e, q);
}

int reduce_received(mox_engine* e, uint64_t rs, uint64_t rb, uint64_t r_long, const XDir& rdir, const mox_stats& local,
                    std::chrono::steady_clock::time_point t0);

// The exchange in three phases, so that one process per GPU (exchange_impl,
// with a Transport) and an engine group (group_exchange, every member's phase
// from one host thread) run the same code:
//   x_begin : per-destination counts of the local table (k_xcount)   [enqueued]
//   ... counts all-to-all (transport) -> h_send / h_recv rows on the host
//   x_pack  : send / receive layout, pack kernels                     [enqueued]
//   ... payload all-to-all (transport) -> x_recv_short / x_recv_blob
//   x_reduce: reduce-only pass over the received partials (synchronous)
struct XPlan {
  int P = 1;
  bool ranged = false;  // sorted exchange (MOX_F_SORT_BYTES): byte-range owners, every rank sorts its words
  XSplit split{};
  uint64_t s_short_off[MAX_RANKS], s_short_len[MAX_RANKS], s_blob_off[MAX_RANKS], s_blob_len[MAX_RANKS];
  uint64_t r_short_off[MAX_RANKS], r_short_len[MAX_RANKS], r_blob_off[MAX_RANKS], r_blob_len[MAX_RANKS];
  uint64_t ns = 0, sb = 0, rs = 0, rb = 0, r_long = 0;
  XDir sdir{}, rdir{};
  mox_stats local{};
  std::chrono::steady_clock::time_point t0;
};

void xplan_free(mox_engine* e) {
  delete e->xp;
  e->xp = nullptr;
}

int x_alloc(mox_engine* e) {
  int rc;
  if (!e->d_xcnt) {
    if ((rc = dalloc(e, (void**)&e->d_xcnt, 2 * MAX_RANKS * sizeof(XCnt)))) return rc;
    if ((rc = dalloc(e, (void**)&e->d_xcur, 3 * MAX_RANKS * 8))) return rc;
    HIPCHK(hipHostMalloc((void**)&e->h_xcnt, 2 * MAX_RANKS * sizeof(XCnt), hipHostMallocDefault));
    HIPCHK(hipHostMalloc((void**)&e->h_ctl_x, sizeof(Ctl), hipHostMallocDefault));
  }
  if (!e->xp) {
    e->xp = new (std::nothrow) XPlan();
    if (!e->xp) return fail(MOX_ENOMEM, "host allocation failed");
  }
  return MOX_OK;
}

// Phase 1: k_xcount into the device send rows d_xcnt[0, P).  Sorted exchange
// (MOX_F_SORT_BYTES): k_xsample instead, this rank's sorted sample block into
// d_xs (one copy per peer); the caller moves every rank's block to every rank
// (d_xr) and calls x_split, which picks the splitters on the device and runs
// k_xcount_r.
int x_begin(mox_engine* e, int P) {
  if (int rc = drain_async(e)) return rc;
  if (!e->have_result || !e->res.pass) return fail(MOX_ESTATE, "no local result: mox_run_range first");
  if (P > MAX_RANKS) return fail(MOX_EINVAL, "at most %d ranks", MAX_RANKS);
  HIPCHK(hipSetDevice(e->device));
  if (int rc = x_alloc(e)) return rc;
  XPlan& x = *e->xp;
  x.P = P;
  x.ranged = (e->flags & MOX_F_SORT_BYTES) != 0;
  x.t0 = std::chrono::steady_clock::now();
  x.local = e->stats;  // the exchange pass reuses the phase events
  HIPCHK(hipMemsetAsync(e->d_xcnt, 0, P * sizeof(XCnt), e->stream));
  if (x.ranged) {
    int rc;
    constexpr size_t SB = (size_t)MAX_RANKS * XS_BLOCK * 8;
    if (!e->d_xs && ((rc = dalloc(e, (void**)&e->d_xs, SB)) || (rc = dalloc(e, (void**)&e->d_xr, SB)) ||
                     (rc = dalloc(e, (void**)&e->d_xsp, MAX_RANKS * 8 + 64))))
      return rc;
    if (!e->h_xflag) HIPCHK(hipHostMalloc((void**)&e->h_xflag, 64, hipHostMallocDefault));
    if (!e->ev_xs) HIPCHK(hipEventCreateWithFlags(&e->ev_xs, hipEventDisableTiming));
    hipLaunchKernelGGL(k_xsample, dim3(1), dim3(XS_SAMPLES), 0, e->stream, e->w, e->d_xs);
    for (int d = 1; d < P; d++)
      HIPCHK(hipMemcpyAsync(e->d_xs + (size_t)d * XS_BLOCK, e->d_xs, XS_BLOCK * 8, hipMemcpyDeviceToDevice, e->stream));
  } else {
    hipLaunchKernelGGL(k_xcount, dim3(64), dim3(256), 0, e->stream, e->w, (uint32_t)P, e->d_xcnt);
  }
  HIPCHK(hipGetLastError());
  return MOX_OK;
}

// Sorted exchange, after every rank's sample block is in d_xr (the same on
// every rank, so every rank picks the same splitters): the weighted splitters
// on the device (k_xsplit), the per-destination counts by range owner
// (k_xcount_r), and the skew flag copied to the host behind them (read after
// the counts all-to-all's synchronisation: no round trip of its own).
int x_split(mox_engine* e) {
  HIPCHK(hipSetDevice(e->device));
  XPlan& x = *e->xp;
  uint32_t* d_flag = reinterpret_cast<uint32_t*>(e->d_xsp + MAX_RANKS);
  hipLaunchKernelGGL(k_xsplit, dim3(1), dim3(1024), 0, e->stream, (const uint64_t*)e->d_xr, (uint32_t)x.P, e->d_xsp, d_flag);
  x.split = XSplit{};
  x.split.P = (uint32_t)x.P;
  x.split.sp = e->d_xsp;
  hipLaunchKernelGGL(k_xcount_r, dim3(1024), dim3(256), 0, e->stream, e->w, x.split, e->d_xcnt);
  HIPCHK(hipGetLastError());
  HIPCHK(hipMemcpyAsync(e->h_xflag, d_flag, 4, hipMemcpyDeviceToHost, e->stream));
  return MOX_OK;
}

// Skewed prefixes (k_xsplit's flag: one 8-byte prefix holds several ranks'
// shares): this exchange falls back to hash owners (the gathered table is then
// sorted at the root, as an unsorted one is).  Every rank reads the same flag.
int x_unrange(mox_engine* e) {
  HIPCHK(hipSetDevice(e->device));
  XPlan& x = *e->xp;
  x.ranged = false;
  HIPCHK(hipMemsetAsync(e->d_xcnt, 0, x.P * sizeof(XCnt), e->stream));
  hipLaunchKernelGGL(k_xcount, dim3(64), dim3(256), 0, e->stream, e->w, (uint32_t)x.P, e->d_xcnt);
  HIPCHK(hipGetLastError());
  return MOX_OK;
}

// Send / receive layout of one rank from its count rows (h_send[d] = what it
// sends to peer d, h_recv[s] = what peer s sends to it): per-peer byte offsets
// and lengths of both payloads, packed in peer order.  Pure host arithmetic;
// rank i's s_*_len[p] equals rank p's r_*_len[i] whenever h_recv is the
// transpose of the ranks' h_send rows (count_transpose, the transports), so
// both sides of every pair skip or post the same send / receive
// (tests/test_exchange_plan.py).
void x_layout(XPlan& x, const XCnt* h_send, const XCnt* h_recv) {
  const int P = x.P;
  x.ns = x.sb = x.rs = x.rb = x.r_long = 0;
  x.sdir = XDir{};
  x.rdir = XDir{};
  x.sdir.P = x.rdir.P = (uint32_t)P;
  for (int d = 0; d < P; d++) {
    x.s_short_off[d] = x.ns * sizeof(WRec);
    x.s_short_len[d] = h_send[d].n_short * sizeof(WRec);
    x.ns += h_send[d].n_short;
    x.sdir.blob[d] = x.s_blob_off[d] = x.sb;
    x.sdir.nlong[d] = h_send[d].n_long;
    x.s_blob_len[d] = h_send[d].n_long * sizeof(XHdr) + h_send[d].long_bytes;
    x.sb += x.s_blob_len[d];
    x.r_short_off[d] = x.rs * sizeof(WRec);
    x.r_short_len[d] = h_recv[d].n_short * sizeof(WRec);
    x.rs += h_recv[d].n_short;
    x.rdir.blob[d] = x.r_blob_off[d] = x.rb;
    x.rdir.nlong[d] = h_recv[d].n_long;
    x.rdir.hpre[d] = x.r_long;
    x.r_long += h_recv[d].n_long;
    x.r_blob_len[d] = h_recv[d].n_long * sizeof(XHdr) + h_recv[d].long_bytes;
    x.rb += x.r_blob_len[d];
  }
  x.sdir.blob[P] = x.sb;
  x.rdir.blob[P] = x.rb;
  x.rdir.hpre[P] = x.r_long;
}

// The count all-to-all of the device-copy transport (and its model in the
// test hook): member i's receive row s = member s's send row i.
void count_transpose(int P, XCnt* const* send_rows, XCnt* const* recv_rows) {
  for (int i = 0; i < P; i++)
    for (int s = 0; s < P; s++) recv_rows[i][s] = send_rows[s][i];
}

// Phase 2: layout from the host count rows (h_xcnt[0, P) = what this rank
// sends to each peer, h_xcnt[MAX_RANKS + s] = what peer s sends here), then
// the pack kernels into x_send_short / x_send_blob.
int x_pack(mox_engine* e) {
  HIPCHK(hipSetDevice(e->device));
  XPlan& x = *e->xp;
  const int P = x.P;
  x_layout(x, e->h_xcnt, e->h_xcnt + MAX_RANKS);
  int rc;
  if ((rc = grow_dev(e->x_send_short, x.ns * sizeof(WRec) + 64)) || (rc = grow_dev(e->x_send_blob, x.sb + 64)) ||
      (rc = grow_dev(e->x_recv_short, x.rs * sizeof(WRec) + 64)) || (rc = grow_dev(e->x_recv_blob, x.rb + 64)))
    return rc;
  hipStream_t s = e->stream;
  if (x.ranged) {
    for (int d = 0; d < P; d++) x.split.soff[d] = x.s_short_off[d] / sizeof(WRec);
    HIPCHK(hipMemsetAsync(e->d_xcur, 0, 3 * MAX_RANKS * 8, s));
    hipLaunchKernelGGL(k_xpack_r, dim3(1024), dim3(256), 0, s, e->w, x.split, x.sdir, e->d_xcur, (WRec*)e->x_send_short.p,
                       (uint8_t*)e->x_send_blob.p);
  } else {
    hipLaunchKernelGGL(k_xpack_short, dim3(1024), dim3(256), 0, s, e->w, (WRec*)e->x_send_short.p);
    HIPCHK(hipMemsetAsync(e->d_xcur, 0, 2 * MAX_RANKS * 8, s));
    hipLaunchKernelGGL(k_xpack_long, dim3(256), dim3(256), 0, s, e->w, x.sdir, e->d_xcur, (uint8_t*)e->x_send_blob.p);
  }
  HIPCHK(hipGetLastError());
  return MOX_OK;
}

// Phase 3: the reduce-only pass over the received partials (the local table
// is no longer needed: buffers may be regrown).  Afterwards this rank owns the
// final counts of its words.
// Sorted exchange: this rank's words are a byte range, sorted here (its own
// GPU, in parallel with the other ranks), so the gather in rank order is the
// sorted table.  A table the device sort cannot take stays in engine order
// (the gathered table is then sorted where it is fetched).
int x_reduce(mox_engine* e) {
  HIPCHK(hipSetDevice(e->device));
  const XPlan& x = *e->xp;
  if (int rc = reduce_received(e, x.rs, x.rb, x.r_long, x.rdir, x.local, x.t0)) return rc;
  e->stats.x_bytes_sent = x.ns * sizeof(WRec) + x.sb + x.P * sizeof(XCnt) + (x.ranged ? x.P * XS_BLOCK * 8 : 0);
  e->stats.x_bytes_recv = x.rs * sizeof(WRec) + x.rb + x.P * sizeof(XCnt) + (x.ranged ? x.P * XS_BLOCK * 8 : 0);
  e->res.exchanged = true;
  e->stats.x_ranged = x.ranged ? 1u : 0u;
  if (x.ranged) {
    const auto t0 = std::chrono::steady_clock::now();
    const int rc = bsort_table(e);
    if (rc != MOX_OK && rc != MOX_ENOMEM) return rc;
    e->stats.ms_sort = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  }
  return MOX_OK;
}

int exchange_impl(mox_engine* e, int P, int me, Transport& T) {
  (void)me;
  int rc;
  if ((rc = x_begin(e, P))) return rc;
  if (e->xp->ranged) {  // every rank's sample block to every rank, then the splitters on the device
    uint64_t off[MAX_RANKS], len[MAX_RANKS];
    for (int d = 0; d < P; d++) {
      off[d] = (uint64_t)d * XS_BLOCK * 8;
      len[d] = XS_BLOCK * 8;
    }
    if ((rc = T.alltoallv((const uint8_t*)e->d_xs, off, len, (uint8_t*)e->d_xr, off, len))) return rc;
    if ((rc = x_split(e))) return rc;
  }
  if ((rc = T.counts(e->d_xcnt, e->d_xcnt + MAX_RANKS, e->h_xcnt, e->h_xcnt + MAX_RANKS))) return rc;
  if (e->xp->ranged && *e->h_xflag) {  // skewed prefixes: hash owners (the same decision on every rank)
    if ((rc = x_unrange(e))) return rc;
    if ((rc = T.counts(e->d_xcnt, e->d_xcnt + MAX_RANKS, e->h_xcnt, e->h_xcnt + MAX_RANKS))) return rc;
  }
  if ((rc = x_pack(e))) return rc;
  const XPlan& x = *e->xp;
  if ((rc = T.alltoallv_pair((const uint8_t*)e->x_send_short.p, x.s_short_off, x.s_short_len, (uint8_t*)e->x_recv_short.p,
                             x.r_short_off, x.r_short_len, (const uint8_t*)e->x_send_blob.p, x.s_blob_off, x.s_blob_len,
                             (uint8_t*)e->x_recv_blob.p, x.r_blob_off, x.r_blob_len)))
    return rc;
  return x_reduce(e);
}

// ============================================================== gather (mox_gather)
// Every rank sends its final table [counts (8 n) | offs (8 n) | bytes (nb,
// padded to 8)] to the root; the root concatenates the blocks in rank order
// (counts and bytes by device copies, offsets rebased by k_gather_offs) into
// its gather buffers, which then become its result.  Ranks own disjoint words
// after the exchange, so the concatenation is the whole corpus's table.
// Only an exchanged table can be gathered: after a plain local
// pass the ranks' tables overlap, and a gathered table is not gathered again.
int gather_check(mox_engine* e, int P, int root) {
  if (int rc = drain_async(e)) return rc;
  if (!e->have_result) return fail(MOX_ESTATE, "no result to gather: run (and exchange) first");
  if (P > MAX_RANKS || root < 0 || root >= P) return fail(MOX_EINVAL, "bad root %d of %d ranks", root, P);
  if (P > 1 && !e->res.exchanged)
    return fail(MOX_ESTATE, "gather needs the table of an exchange (mox_exchange first; a gathered table is final)");
  return MOX_OK;
}

int gather_impl(mox_engine* e, int P, int me, int root, Transport& T) {
  if (int rc = gather_check(e, P, root)) return rc;
  HIPCHK(hipSetDevice(e->device));
  hipStream_t s = e->stream;
  int rc;
  const auto t0 = std::chrono::steady_clock::now();
  if ((rc = x_alloc(e))) return rc;
  const mox_engine::Res r = e->res;
  const uint64_t n = r.n, nb = r.nb, nb8 = (nb + 7) & ~7ull, block = 16 * n + nb8;
  // 1. sizes: every rank's (n, nb, tokens) row to every peer (only the root uses them)
  XCnt* d_send = e->d_xcnt;
  XCnt* d_recv = e->d_xcnt + MAX_RANKS;
  XCnt* h_send = e->h_xcnt;
  XCnt* h_recv = e->h_xcnt + MAX_RANKS;
  for (int d = 0; d < P; d++) h_send[d] = XCnt{n, nb, r.tokens, r.sorted ? 1ull : 0ull};  // pad: this rank's table is sorted
  HIPCHK(hipMemcpyAsync(d_send, h_send, P * sizeof(XCnt), hipMemcpyHostToDevice, s));
  if ((rc = T.counts(d_send, d_recv, h_send, h_recv))) return rc;
  // 2. this rank's block -> the root
  if ((rc = grow_dev(e->x_send_blob, block + 64))) return rc;
  uint8_t* sb = (uint8_t*)e->x_send_blob.p;
  if (n) {
    HIPCHK(hipMemcpyAsync(sb, r.counts, 8 * n, hipMemcpyDeviceToDevice, s));
    HIPCHK(hipMemcpyAsync(sb + 8 * n, r.offs, 8 * n, hipMemcpyDeviceToDevice, s));
    if (nb) HIPCHK(hipMemcpyAsync(sb + 16 * n, r.bytes, nb, hipMemcpyDeviceToDevice, s));
  }
  uint64_t soff[MAX_RANKS], slen[MAX_RANKS], roff[MAX_RANKS], rlen[MAX_RANKS];
  uint64_t so = 0, ro = 0, N = 0, NBt = 0, tok = 0;
  bool all_sorted = true;  // every rank sorted its byte range (sorted exchange): the concatenation is sorted
  GDir gd{};
  gd.P = (uint32_t)P;
  for (int d = 0; d < P; d++) {
    soff[d] = so;
    slen[d] = d == root ? block : 0;
    so += slen[d];
    const uint64_t bn = h_recv[d].n_short, bb = h_recv[d].n_long;  // rank d's n, nb
    roff[d] = ro;
    rlen[d] = me == root ? 16 * bn + ((bb + 7) & ~7ull) : 0;
    gd.roff[d] = ro + 8 * bn;  // rank d's offs block
    gd.base_n[d] = N;
    gd.base_b[d] = NBt;
    ro += rlen[d];
    N += bn;
    NBt += bb;
    tok += h_recv[d].long_bytes;
    all_sorted = all_sorted && h_recv[d].pad != 0;
  }
  gd.base_n[P] = N;
  gd.base_b_total = NBt;
  if (me == root && (rc = grow_dev(e->g_recv, ro + 64))) return rc;
  if ((rc = T.alltoallv(sb, soff, slen, (uint8_t*)(me == root ? e->g_recv.p : e->x_send_blob.p), roff, rlen))) return rc;
  e->stats.gather_bytes = me == root ? ro : block;
  if (me == root) {
    // 3. root: concatenate in rank order
    if ((rc = grow_dev(e->g_counts, 8 * N + 64)) || (rc = grow_dev(e->g_offs, 8 * (N + 1) + 64)) ||
        (rc = grow_dev(e->g_bytes, NBt + 64)))
      return rc;
    const uint8_t* rb = (const uint8_t*)e->g_recv.p;
    for (int d = 0; d < P; d++) {
      const uint64_t bn = h_recv[d].n_short, bb = h_recv[d].n_long;
      if (bn) HIPCHK(hipMemcpyAsync((uint64_t*)e->g_counts.p + gd.base_n[d], rb + roff[d], 8 * bn, hipMemcpyDeviceToDevice, s));
      if (bb) HIPCHK(hipMemcpyAsync((uint8_t*)e->g_bytes.p + gd.base_b[d], rb + roff[d] + 16 * bn, bb, hipMemcpyDeviceToDevice, s));
    }
    hipLaunchKernelGGL(k_gather_offs, dim3(256), dim3(256), 0, s, rb, gd, (uint64_t*)e->g_offs.p);
    HIPCHK(hipGetLastError());
    HIPCHK(hipStreamSynchronize(s));
    e->res.counts = (const uint64_t*)e->g_counts.p;
    e->res.offs = (const uint64_t*)e->g_offs.p;
    e->res.bytes = (const uint8_t*)e->g_bytes.p;
    e->res.n = N;
    e->res.nb = NBt;
    e->res.tokens = tok;
    e->res.pass = false;
    e->res.exchanged = false;  // gathered: final, not gathered again
    e->res.sorted = all_sorted && e->xp && e->xp->ranged;
  } else {
    HIPCHK(hipStreamSynchronize(s));  // the send buffer is reused by the next exchange
    e->res.exchanged = false;  // sent to the root: a table takes part in one gather
  }
  e->stats.ms_gather = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  return MOX_OK;
}

// ============================================================== engine group
// (mox_config.n_gpus > 1; SURVEY.md §8(b): one engine for n GPUs, driven from
// the calling thread.)  Member 0 is the engine the caller holds; the others
// are plain engines on their own devices.  A call runs:
//   1. the local passes of all members at once (one worker thread per member
//      for the host side of the pass; the GPUs run concurrently);
//   2. the exchange: x_begin on every member, the counts and payload
//      all-to-alls as ONE ncclGroupStart/End each over the members'
//      communicators (ncclCommInitAll; MOX_XPORT_RCCL) or as device-to-device
//      copies (MOX_XPORT_COPY), then x_reduce on every member at once;
//   3. the gather of every member's final table straight into member 0's
//      gather buffers (counts and bytes at their final place, offsets rebased
//      by k_gather_offs): RCCL send/recv or peer copies;
//   4. with MOX_F_SORT_BYTES, the bytewise sort of the gathered table on
//      member 0's GPU (mox_bsort.hip).
struct Group {
  int n = 1;
  uint32_t xport = MOX_XPORT_RCCL;
  std::vector<mox_engine*> m;     // m[0] = the owning engine
  std::vector<ncclComm_t> comms;  // MOX_XPORT_RCCL: member i's communicator (rank i)
};

// f(i) for every member at once, each on a thread of its own (current device
// set to the member's); returns the first failing member's status and message.
template <class F>
int for_members(Group& G, F f) {
  std::vector<int> rc(G.n, MOX_OK);
  std::vector<std::string> msg(G.n);
  std::vector<std::thread> th;
  th.reserve(G.n);
  for (int i = 0; i < G.n; i++)
    th.emplace_back([&, i] {
      if (hipSetDevice(G.m[i]->device) != hipSuccess) { rc[i] = MOX_EHIP; msg[i] = "hipSetDevice failed"; return; }
      rc[i] = f(i);
      if (rc[i]) msg[i] = g_err;
    });
  for (auto& t : th) t.join();
  for (int i = 0; i < G.n; i++)
    if (rc[i]) {
      g_err = "member " + std::to_string(i) + ": " + msg[i];
      return rc[i];
    }
  return MOX_OK;
}

int sync_members(Group& G) {
  for (int i = 0; i < G.n; i++) {
    HIPCHK(hipSetDevice(G.m[i]->device));
    HIPCHK(hipStreamSynchronize(G.m[i]->stream));
  }
  return MOX_OK;
}

void group_destroy(mox_engine* e) {
  Group* G = e->grp;
  if (!G) return;
  e->grp = nullptr;
  for (ncclComm_t c : G->comms)
    if (c) ncclCommDestroy(c);
  for (int i = 1; i < G->n; i++) mox_engine_destroy(G->m[i]);
  delete G;
}

int group_create(mox_engine* e, const mox_config* cfg) {
  Group* G = new (std::nothrow) Group();
  if (!G) return fail(MOX_ENOMEM, "host allocation failed");
  e->grp = G;
  G->n = (int)cfg->n_gpus;
  G->xport = cfg->transport;
  if (G->xport != MOX_XPORT_RCCL && G->xport != MOX_XPORT_COPY) return fail(MOX_EINVAL, "unknown transport %u", G->xport);
  std::vector<int> dev(G->n);
  for (int i = 0; i < G->n; i++) dev[i] = cfg->n_devices ? cfg->devices[i] : i;
  dev[0] = e->device;
  G->m.assign(G->n, nullptr);
  G->m[0] = e;
  for (int i = 1; i < G->n; i++) {
    if (int rc = engine_create_one(cfg, dev[i], &G->m[i])) return rc;  // group_destroy frees the members made so far
  }
  if (G->xport == MOX_XPORT_RCCL) {
    for (int i = 0; i < G->n; i++)
      for (int j = 0; j < i; j++)
        if (dev[i] == dev[j])
          return fail(MOX_EINVAL, "RCCL transport: members %d and %d share device %d (use MOX_XPORT_COPY)", j, i, dev[i]);
    G->comms.assign(G->n, nullptr);
    RCCLCHK(ncclCommInitAll(G->comms.data(), G->n, dev.data()));
    for (int i = 0; i < G->n; i++) {
      G->m[i]->nranks = G->n;
      G->m[i]->rank = i;
    }
  } else {
    // peer access between distinct devices (xGMI); already-enabled is fine
    for (int i = 0; i < G->n; i++)
      for (int j = 0; j < G->n; j++)
        if (dev[i] != dev[j]) {
          int ok = 0;
          if (hipDeviceCanAccessPeer(&ok, dev[i], dev[j]) == hipSuccess && ok) {
            (void)hipSetDevice(dev[i]);
            (void)hipDeviceEnablePeerAccess(dev[j], 0);
            (void)hipGetLastError();
          }
        }
  }
  return MOX_OK;
}

// Phase 2 of the exchange for the whole group: the count rows.
int group_counts(Group& G) {
  const int P = G.n;
  if (G.xport == MOX_XPORT_RCCL) {
    RCCLCHK(ncclGroupStart());
    for (int i = 0; i < P; i++) {
      mox_engine* e = G.m[i];
      for (int p = 0; p < P; p++) {
        RCCLCHK(ncclSend(e->d_xcnt + p, sizeof(XCnt), ncclUint8, p, G.comms[i], e->stream));
        RCCLCHK(ncclRecv(e->d_xcnt + MAX_RANKS + p, sizeof(XCnt), ncclUint8, p, G.comms[i], e->stream));
      }
    }
    RCCLCHK(ncclGroupEnd());
    for (int i = 0; i < P; i++) {
      mox_engine* e = G.m[i];
      HIPCHK(hipSetDevice(e->device));
      HIPCHK(hipMemcpyAsync(e->h_xcnt, e->d_xcnt, 2 * MAX_RANKS * sizeof(XCnt), hipMemcpyDeviceToHost, e->stream));
    }
    return sync_members(G);
  }
  for (int i = 0; i < P; i++) {
    mox_engine* e = G.m[i];
    HIPCHK(hipSetDevice(e->device));
    HIPCHK(hipMemcpyAsync(e->h_xcnt, e->d_xcnt, P * sizeof(XCnt), hipMemcpyDeviceToHost, e->stream));
  }
  if (int rc = sync_members(G)) return rc;
  std::vector<XCnt*> snd(P), rcv(P);
  for (int i = 0; i < P; i++) {
    snd[i] = G.m[i]->h_xcnt;
    rcv[i] = G.m[i]->h_xcnt + MAX_RANKS;
  }
  count_transpose(P, snd.data(), rcv.data());
  return MOX_OK;
}

// Sorted exchange, the whole group: member i's sample block (d_xs) into every
// member's d_xr block i, device to device with no host synchronisation (RCCL
// send / recv in one group, or peer copies ordered after the sender's
// k_xsample by an event).
int group_samples(Group& G) {
  const int P = G.n;
  constexpr size_t BB = XS_BLOCK * 8;
  if (G.xport == MOX_XPORT_RCCL) {
    RCCLCHK(ncclGroupStart());
    for (int i = 0; i < P; i++) {
      mox_engine* e = G.m[i];
      for (int p = 0; p < P; p++) {
        RCCLCHK(ncclSend(e->d_xs + (size_t)p * XS_BLOCK, BB, ncclUint8, p, G.comms[i], e->stream));
        RCCLCHK(ncclRecv(e->d_xr + (size_t)p * XS_BLOCK, BB, ncclUint8, p, G.comms[i], e->stream));
      }
    }
    RCCLCHK(ncclGroupEnd());
    return MOX_OK;
  }
  for (int i = 0; i < P; i++) {
    HIPCHK(hipSetDevice(G.m[i]->device));
    HIPCHK(hipEventRecord(G.m[i]->ev_xs, G.m[i]->stream));
  }
  for (int j = 0; j < P; j++) {
    mox_engine* r = G.m[j];
    HIPCHK(hipSetDevice(r->device));
    for (int i = 0; i < P; i++) {
      const mox_engine* snd = G.m[i];
      HIPCHK(hipStreamWaitEvent(r->stream, snd->ev_xs, 0));
      HIPCHK(hipMemcpyPeerAsync(r->d_xr + (size_t)i * XS_BLOCK, r->device, snd->d_xs, snd->device, BB, r->stream));
    }
  }
  return MOX_OK;
}

// Phase 2' of the exchange for the whole group: both payloads.
int group_payloads(Group& G) {
  const int P = G.n;
  if (G.xport == MOX_XPORT_RCCL) {
    for (int i = 0; i < P; i++) {  // self blocks: device copies
      mox_engine* e = G.m[i];
      const XPlan& x = *e->xp;
      HIPCHK(hipSetDevice(e->device));
      if (x.s_short_len[i])
        HIPCHK(hipMemcpyAsync((uint8_t*)e->x_recv_short.p + x.r_short_off[i], (const uint8_t*)e->x_send_short.p + x.s_short_off[i],
                              x.s_short_len[i], hipMemcpyDeviceToDevice, e->stream));
      if (x.s_blob_len[i])
        HIPCHK(hipMemcpyAsync((uint8_t*)e->x_recv_blob.p + x.r_blob_off[i], (const uint8_t*)e->x_send_blob.p + x.s_blob_off[i],
                              x.s_blob_len[i], hipMemcpyDeviceToDevice, e->stream));
    }
    RCCLCHK(ncclGroupStart());
    for (int i = 0; i < P; i++) {
      mox_engine* e = G.m[i];
      const XPlan& x = *e->xp;
      for (int p = 0; p < P; p++) {
        if (p == i) continue;
        if (x.s_short_len[p])
          RCCLCHK(ncclSend((const uint8_t*)e->x_send_short.p + x.s_short_off[p], x.s_short_len[p], ncclUint8, p, G.comms[i], e->stream));
        if (x.r_short_len[p])
          RCCLCHK(ncclRecv((uint8_t*)e->x_recv_short.p + x.r_short_off[p], x.r_short_len[p], ncclUint8, p, G.comms[i], e->stream));
        if (x.s_blob_len[p])
          RCCLCHK(ncclSend((const uint8_t*)e->x_send_blob.p + x.s_blob_off[p], x.s_blob_len[p], ncclUint8, p, G.comms[i], e->stream));
        if (x.r_blob_len[p])
          RCCLCHK(ncclRecv((uint8_t*)e->x_recv_blob.p + x.r_blob_off[p], x.r_blob_len[p], ncclUint8, p, G.comms[i], e->stream));
      }
    }
    RCCLCHK(ncclGroupEnd());
    return MOX_OK;
  }
  // copies: every sender's pack must be complete before its peers read
  if (int rc = sync_members(G)) return rc;
  for (int i = 0; i < P; i++) {
    mox_engine* r = G.m[i];
    const XPlan& xr = *r->xp;
    HIPCHK(hipSetDevice(r->device));
    for (int s = 0; s < P; s++) {
      const mox_engine* snd = G.m[s];
      const XPlan& xs = *snd->xp;
      if (xs.s_short_len[i])
        HIPCHK(hipMemcpyPeerAsync((uint8_t*)r->x_recv_short.p + xr.r_short_off[s], r->device,
                                  (const uint8_t*)snd->x_send_short.p + xs.s_short_off[i], snd->device, xs.s_short_len[i], r->stream));
      if (xs.s_blob_len[i])
        HIPCHK(hipMemcpyPeerAsync((uint8_t*)r->x_recv_blob.p + xr.r_blob_off[s], r->device,
                                  (const uint8_t*)snd->x_send_blob.p + xs.s_blob_off[i], snd->device, xs.s_blob_len[i], r->stream));
    }
  }
  return MOX_OK;
}

int group_exchange(Group& G) {
  const int P = G.n;
  for (int i = 0; i < P; i++)
    if (int rc = x_begin(G.m[i], P)) return rc;
  if (G.m[0]->xp->ranged) {  // sorted exchange: every member's sample block to every member, splitters on each GPU
    if (int rc = group_samples(G)) return rc;
    for (int i = 0; i < P; i++)
      if (int rc = x_split(G.m[i])) return rc;
  }
  if (int rc = group_counts(G)) return rc;
  if (G.m[0]->xp->ranged && *G.m[0]->h_xflag) {  // skewed prefixes: hash owners on every member
    for (int i = 0; i < P; i++)
      if (int rc = x_unrange(G.m[i])) return rc;
    if (int rc = group_counts(G)) return rc;
  }
  for (int i = 0; i < P; i++)
    if (int rc = x_pack(G.m[i])) return rc;
  if (int rc = group_payloads(G)) return rc;
  return for_members(G, [&](int i) { return x_reduce(G.m[i]); });
}

// Every member's final table into member 0's gather buffers.
int group_gather(Group& G) {
  const int P = G.n;
  mox_engine* root = G.m[0];
  uint64_t N = 0, NBt = 0, tok = 0, recv_bytes = 0;
  bool all_sorted = root->xp && root->xp->ranged;  // sorted exchange: the members' sorted ranges in member order
  GDir gd{};
  gd.P = (uint32_t)P;
  for (int i = 0; i < P; i++) {
    const auto& r = G.m[i]->res;
    if (!r.exchanged) return fail(MOX_ESTATE, "member %d has no exchanged table", i);
    all_sorted = all_sorted && r.sorted;
    gd.roff[i] = 8 * N;  // member i's offsets inside g_recv
    gd.base_n[i] = N;
    gd.base_b[i] = NBt;
    N += r.n;
    NBt += r.nb;
    tok += r.tokens;
    if (i) recv_bytes += 16 * r.n + r.nb;
  }
  gd.base_n[P] = N;
  gd.base_b_total = NBt;
  HIPCHK(hipSetDevice(root->device));
  int rc;
  if ((rc = grow_dev(root->g_counts, 8 * N + 64)) || (rc = grow_dev(root->g_offs, 8 * (N + 1) + 64)) ||
      (rc = grow_dev(root->g_bytes, NBt + 64)) || (rc = grow_dev(root->g_recv, 8 * N + 64)))
    return rc;
  uint64_t* gc = (uint64_t*)root->g_counts.p;
  uint8_t* gb = (uint8_t*)root->g_bytes.p;
  uint8_t* go = (uint8_t*)root->g_recv.p;
  const auto& r0 = root->res;
  hipStream_t s0 = root->stream;
  if (r0.n) {
    HIPCHK(hipMemcpyAsync(gc, r0.counts, 8 * r0.n, hipMemcpyDeviceToDevice, s0));
    HIPCHK(hipMemcpyAsync(go, r0.offs, 8 * r0.n, hipMemcpyDeviceToDevice, s0));
    if (r0.nb) HIPCHK(hipMemcpyAsync(gb, r0.bytes, r0.nb, hipMemcpyDeviceToDevice, s0));
  }
  if (G.xport == MOX_XPORT_RCCL) {
    RCCLCHK(ncclGroupStart());
    for (int i = 1; i < P; i++) {
      mox_engine* e = G.m[i];
      const auto& r = e->res;
      if (!r.n) continue;
      RCCLCHK(ncclSend(r.counts, 8 * r.n, ncclUint8, 0, G.comms[i], e->stream));
      RCCLCHK(ncclRecv(gc + gd.base_n[i], 8 * r.n, ncclUint8, i, G.comms[0], s0));
      RCCLCHK(ncclSend(r.offs, 8 * r.n, ncclUint8, 0, G.comms[i], e->stream));
      RCCLCHK(ncclRecv(go + gd.roff[i], 8 * r.n, ncclUint8, i, G.comms[0], s0));
      if (r.nb) {
        RCCLCHK(ncclSend(r.bytes, r.nb, ncclUint8, 0, G.comms[i], e->stream));
        RCCLCHK(ncclRecv(gb + gd.base_b[i], r.nb, ncclUint8, i, G.comms[0], s0));
      }
    }
    RCCLCHK(ncclGroupEnd());
  } else {
    for (int i = 1; i < P; i++) {  // the members' tables are complete (x_reduce synchronised)
      const mox_engine* e = G.m[i];
      const auto& r = e->res;
      if (!r.n) continue;
      HIPCHK(hipMemcpyPeerAsync(gc + gd.base_n[i], root->device, r.counts, e->device, 8 * r.n, s0));
      HIPCHK(hipMemcpyPeerAsync(go + gd.roff[i], root->device, r.offs, e->device, 8 * r.n, s0));
      if (r.nb) HIPCHK(hipMemcpyPeerAsync(gb + gd.base_b[i], root->device, r.bytes, e->device, r.nb, s0));
    }
  }
  HIPCHK(hipSetDevice(root->device));
  hipLaunchKernelGGL(k_gather_offs, dim3(256), dim3(256), 0, s0, (const uint8_t*)go, gd, (uint64_t*)root->g_offs.p);
  HIPCHK(hipGetLastError());
  if (int rc2 = sync_members(G)) return rc2;
  auto& res = root->res;
  res.counts = gc;
  res.offs = (const uint64_t*)root->g_offs.p;
  res.bytes = gb;
  res.n = N;
  res.nb = NBt;
  res.tokens = tok;
  res.pass = false;
  res.exchanged = false;
  res.sorted = all_sorted;
  root->have_result = true;
  root->stats.gather_bytes = recv_bytes;
  return MOX_OK;
}

double ms_since(std::chrono::steady_clock::time_point t0) {
  return std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
}

// One group call over per-member corpora c[i] (already on the members' GPUs);
// base[i] = where member i's bytes start in the caller's input (error offsets).
int group_run(mox_engine* e, const std::vector<Corpus>& c, const std::vector<uint64_t>& base = {}) {
  Group& G = *e->grp;
  const auto t0 = std::chrono::steady_clock::now();
  int rc = for_members(G, [&](int i) { return run_corpus(G.m[i], c[i]); });
  if (rc == MOX_EUTF8 && !base.empty()) {  // the reference's InvalidData: report the input offset
    for (int i = 0; i < G.n; i++) {
      const Ctl& h = *G.m[i]->h_ctl;
      if (h.err_utf8 != ~0ull) {
        const uint64_t own = c[i].own_lo - c[i].lo;
        return fail(MOX_EUTF8, "stream did not contain valid UTF-8 (byte %llu)", (unsigned long long)(base[i] + h.err_utf8 - own));
      }
    }
  }
  if (rc) return rc;
  const double ms_local = ms_since(t0);
  uint64_t bytes = 0, tokens = 0, cold = 0, words_local = 0;
  double ms_map = 0;
  for (int i = 0; i < G.n; i++) {
    bytes += G.m[i]->stats.bytes;
    tokens += G.m[i]->stats.tokens;
    cold += G.m[i]->stats.cold_records;
    words_local += G.m[i]->stats.uniques;
    ms_map += G.m[i]->stats.ms_map / G.n;  // MOX_F_TIMING(_MAP): the members' mean map-kernel time
  }
  if ((rc = group_exchange(G))) return rc;
  // the exchange without the sorted exchange's bytewise sorts (reported as
  // ms_sort), as one rank's mox_exchange reports it: the slowest member's
  // time from its x_begin to the end of its reduce pass (reduce_received)
  double ms_x = 0;
  for (int i = 0; i < G.n; i++) ms_x = std::max(ms_x, G.m[i]->stats.ms_exchange);
  uint64_t xs = 0, xr = 0;
  for (int i = 0; i < G.n; i++) {
    xs += G.m[i]->stats.x_bytes_sent;
    xr += G.m[i]->stats.x_bytes_recv;
  }
  const auto t2 = std::chrono::steady_clock::now();
  if ((rc = group_gather(G))) return rc;
  const double ms_g = ms_since(t2);
  double ms_s = 0;
  if (e->flags & MOX_F_SORT_BYTES) {
    if (e->res.sorted) {
      // sorted exchange: every member sorted its byte range on its own GPU
      // inside the exchange; the slowest member's sort
      for (int i = 0; i < G.n; i++) ms_s = std::max(ms_s, G.m[i]->stats.ms_sort);
    } else {
      // a table too big for the sort's device scratch stays in engine order here:
      // mox_fetch_table then sorts it on the host, as for one engine
      const auto t3 = std::chrono::steady_clock::now();
      rc = bsort_table(e);
      if (rc != MOX_OK && rc != MOX_ENOMEM) return rc;
      ms_s = ms_since(t3);
    }
  }
  mox_stats& st = e->stats;  // member 0's pass stats are replaced by the group's
  const uint64_t gb = st.gather_bytes;
  std::memset(&st, 0, sizeof st);
  st.bytes = bytes;
  st.tokens = tokens;
  st.uniques = e->res.n;
  st.cold_records = cold;
  st.weighted_records = words_local;
  st.ms_local = ms_local;
  st.ms_map = ms_map;
  st.ms_exchange = ms_x;
  st.ms_gather = ms_g;
  st.ms_sort = ms_s;
  st.ms_run = ms_since(t0);
  st.x_bytes_sent = xs;
  st.x_bytes_recv = xr;
  st.gather_bytes = gb;
  st.n_gpus = (uint32_t)G.n;
  for (int i = 0; i < G.n; i++)
    for (int k = 0; k < PATH_N; k++) st.path_hits[k] += G.m[i]->stats.path_hits[k];
  if (tokens != e->res.tokens)
    return fail(MOX_EHIP, "engine group: gathered %llu tokens, local passes counted %llu", (unsigned long long)e->res.tokens,
                (unsigned long long)tokens);
  return MOX_OK;
}

// Byte cuts of an input split into n ranges at ASCII whitespace: cut k is the
// first position >= k len / n right after a whitespace byte (or len), so
// every range starts at a token start and ends after a delimiter, no UTF-8
// sequence or multi-byte whitespace straddles a cut, and each range is a
// complete corpus of its own (no halo).  byte_at(p) reads position p.
template <class B>
std::vector<uint64_t> ws_cuts(uint64_t len, int n, B byte_at) {
  std::vector<uint64_t> cut(n + 1, len);
  cut[0] = 0;
  for (int k = 1; k < n; k++) {
    uint64_t p = std::max<uint64_t>(cut[k - 1], len / n * k);
    while (p < len && p > 0) {
      const int b = byte_at(p - 1);
      if (b < 0) { p = len; break; }  // read error: the rest is one range
      if (b == ' ' || (b >= 9 && b <= 13)) break;
      p++;
    }
    cut[k] = p;
  }
  return cut;
}

int group_count_host(mox_engine* e, const uint8_t* text, size_t len) {
  Group& G = *e->grp;
  const std::vector<uint64_t> cut = ws_cuts(len, G.n, [&](uint64_t p) { return (int)text[p]; });
  int rc = for_members(G, [&](int i) { return stage_host_range(G.m[i], text + cut[i], cut[i + 1] - cut[i]); });
  if (rc) return rc;
  std::vector<Corpus> c(G.n);
  for (int i = 0; i < G.n; i++) {
    const size_t n = cut[i + 1] - cut[i];
    c[i] = make_corpus(n ? (const void*)G.m[i]->d_text : (const void*)G.m[i]->w.ctl, n, 0, n, 1);
  }
  return group_run(e, c, std::vector<uint64_t>(cut.begin(), cut.end() - 1));
}

// Each member reads its own byte range of the file (its reader threads,
// pinned buffers and streams) into its GPU: 8 x n_gpus reads in flight.
int group_count_file(mox_engine* e, const char* path) {
  Group& G = *e->grp;
  const int fd = open(path, O_RDONLY);
  if (fd < 0) return fail(MOX_EIO, "cannot open %s: %s", path, strerror(errno));
  struct stat st;
  if (fstat(fd, &st) != 0) {
    close(fd);
    return fail(MOX_EIO, "cannot stat %s: %s", path, strerror(errno));
  }
  const uint64_t len = (uint64_t)st.st_size;
  // cut search: 64 KiB windows read forward from each nominal cut
  std::vector<uint8_t> win(1 << 16);
  uint64_t wlo = 0, whi = 0;
  auto byte_at = [&](uint64_t p) -> int {
    if (p < wlo || p >= whi) {
      const ssize_t r = pread(fd, win.data(), win.size(), (off_t)p);
      if (r <= 0) return -1;
      wlo = p;
      whi = p + (uint64_t)r;
    }
    return win[p - wlo];
  };
  const std::vector<uint64_t> cut = ws_cuts(len, G.n, byte_at);
  const auto t0 = std::chrono::steady_clock::now();
  int rc = for_members(G, [&](int i) { return stage_file_range(G.m[i], fd, cut[i], cut[i + 1] - cut[i]); });
  close(fd);
  if (rc) return rc;
  const double ms_ingest = ms_since(t0);
  std::vector<Corpus> c(G.n);
  for (int i = 0; i < G.n; i++) {
    const size_t n = cut[i + 1] - cut[i];
    c[i] = make_corpus(n ? (const void*)G.m[i]->d_text : (const void*)G.m[i]->w.ctl, n, 0, n, 1);
  }
  if ((rc = group_run(e, c, std::vector<uint64_t>(cut.begin(), cut.end() - 1)))) return rc;
  e->stats.ms_h2d = ms_ingest;
  return MOX_OK;
}

int group_run_shards(mox_engine* e, const mox_shard* sh) {
  Group& G = *e->grp;
  std::vector<Corpus> c(G.n);
  for (int i = 0; i < G.n; i++) {
    const mox_shard& s = sh[i];
    if (!s.d_buf && s.buf_len) return fail(MOX_EINVAL, "shard %d: buffer is NULL", i);
    if (s.own_begin > s.own_end || s.own_end > s.buf_len) return fail(MOX_EINVAL, "shard %d: bad own range", i);
    if (s.own_begin > 0 && s.own_begin < 4) return fail(MOX_EINVAL, "shard %d: own_begin must be 0 or >= 4", i);
    c[i] = make_corpus(s.buf_len ? s.d_buf : (const void*)G.m[i]->w.ctl, s.buf_len, s.own_begin, s.own_end, s.at_corpus_end);
  }
  return group_run(e, c);
}

// Reduce-only pass over partial (word, count) records already in
// x_recv_short (rs WRecs) and x_recv_blob (long-word blobs described by rdir):
// the exchange's final reduce and mox_reduce_pairs (spill files) share it.
int reduce_received(mox_engine* e, uint64_t rs, uint64_t rb, uint64_t r_long, const XDir& rdir, const mox_stats& local,
                    std::chrono::steady_clock::time_point t0) {
  Work& w = e->w;
  int rc;
  Caps need = w.cold ? caps_of(w) : initial_caps(1 << 20, e->n_cu);
  need.w_cap = std::max<uint64_t>(need.w_cap, rs + rs / 8 + 1024);
  need.table_cap = std::max<uint64_t>(need.table_cap, rs + r_long + 1024);
  need.bytes_cap = std::max<uint64_t>(need.bytes_cap, rs * 16 + rb + 65536);
  need.long_cap = std::max<uint64_t>(need.long_cap, next_pow2(2 * r_long + 1024));
  need.arena_cap = std::max<uint64_t>(need.arena_cap, rb + 65536);
  e->have_result = false;
  if ((rc = ensure_caps(e, need))) return rc;  // stream-ordered; a regrow synchronises the device itself
  for (int attempt = 0;; attempt++) {
    if ((rc = exchange_pass_once(e, rs, rb, rdir))) return rc;
    const Ctl& h = *e->h_ctl;
    if ((rc = check_failed(h))) return rc;
    if (!h.overflow) break;
    if (h.overflow & OVF_REDUCE) return fail(MOX_ENOMEM, "a reduce partition holds more distinct words than it can split by hash");
    if (attempt >= GROW_RETRIES) return fail(MOX_ENOMEM, "exchange buffer growth did not converge (overflow mask 0x%x)", h.overflow);
    e->stats.retries++;
    if ((rc = ensure_caps(e, grow_for(e, h)))) return rc;
  }
  const Ctl& h = *e->h_ctl;
  const uint32_t retries = e->stats.retries;
  e->stats = local;
  e->stats.retries = retries;
  e->stats.tokens = h.tokens;
  e->stats.uniques = h.n_total;
  for (int i = 0; i < PATH_N; i++) e->stats.path_hits[i] += h.paths[i];  // the local pass's + this pass's
  e->stats.ms_exchange =std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
  e->last_corpus = Corpus{};
  e->last_corpus.base = (const uint8_t*)w.ctl;
  set_result(e, h);
  return MOX_OK;
}

// Host (word, count) pairs -> the exchange's receive layout (one source):
// words of 1..16 bytes without a NUL byte become 16-byte zero-padded WRec keys,
// every other word an XHdr + its bytes (padded to 8) in the long blob.  Words
// are taken as given (no lowercasing: reduce_phase sums parts[0] verbatim,
// main.rs:160-162,131-134).
int reduce_pairs_impl(mox_engine* e, const uint8_t* bytes, const uint64_t* offs, const uint64_t* counts, uint64_t n) {
  if (int rc = drain_async(e)) return rc;
  HIPCHK(hipSetDevice(e->device));
  const auto t0 = std::chrono::steady_clock::now();
  std::vector<WRec> shorts;
  std::vector<XHdr> hdrs;
  std::vector<uint8_t> lbytes;
  shorts.reserve(n);
  for (uint64_t i = 0; i < n; i++) {
    const uint64_t a = offs[i], len = offs[i + 1] - offs[i];
    if (offs[i + 1] < a) return fail(MOX_EINVAL, "offs not ascending at %llu", (unsigned long long)i);
    if (len == 0) return fail(MOX_EINVAL, "empty word at %llu (split_whitespace never yields one)", (unsigned long long)i);
    const bool nul = memchr(bytes + a, 0, len) != nullptr;
    if (len <= 16 && !nul) {
      uint8_t k[16] = {0};
      memcpy(k, bytes + a, len);
      WRec r;
      memcpy(&r.w0, k, 8);
      memcpy(&r.w1, k + 8, 8);
      r.count = counts[i];
      shorts.push_back(r);
    } else {
      uint64_t h = 0xcbf29ce484222325ull;  // FNV-1a 64 (any hash works: all long words of this pass use it)
      for (uint64_t j = 0; j < len; j++) h = (h ^ bytes[a + j]) * 0x100000001b3ull;
      h = fnv_finish(h);
      hdrs.push_back(XHdr{h, len, counts[i], (uint64_t)lbytes.size()});
      lbytes.insert(lbytes.end(), bytes + a, bytes + a + len);
      lbytes.resize((lbytes.size() + 7) & ~size_t(7), 0);
    }
  }
  const uint64_t rs = shorts.size(), r_long = hdrs.size();
  const uint64_t rb = r_long * sizeof(XHdr) + lbytes.size();
  int rc;
  if ((rc = grow_dev(e->x_recv_short, rs * sizeof(WRec) + 64)) || (rc = grow_dev(e->x_recv_blob, rb + 64))) return rc;
  if (rs) HIPCHK(hipMemcpyAsync(e->x_recv_short.p, shorts.data(), rs * sizeof(WRec), hipMemcpyHostToDevice, e->stream));
  if (r_long) {
    HIPCHK(hipMemcpyAsync(e->x_recv_blob.p, hdrs.data(), r_long * sizeof(XHdr), hipMemcpyHostToDevice, e->stream));
    if (!lbytes.empty())
      HIPCHK(hipMemcpyAsync((uint8_t*)e->x_recv_blob.p + r_long * sizeof(XHdr), lbytes.data(), lbytes.size(),
                            hipMemcpyHostToDevice, e->stream));
  }
  // pageable sources: complete the copies before the vectors go away
  HIPCHK(hipStreamSynchronize(e->stream));
  XDir rdir{};
  rdir.P = 1;
  rdir.blob[0] = 0;
  rdir.blob[1] = rb;
  rdir.nlong[0] = r_long;
  rdir.hpre[0] = 0;
  rdir.hpre[1] = r_long;
  mox_stats local{};
  local.weighted_records = rs + r_long;
  return reduce_received(e, rs, rb, r_long, rdir, local, t0);
}

}  // namespace mox_host

extern "C" {

// ---- multi-GPU ----
int mox_comm_unique_id(uint8_t id[MOX_UNIQUE_ID_BYTES]) {
  if (!id) return fail(MOX_EINVAL, "NULL argument");
  static_assert(sizeof(ncclUniqueId) <= MOX_UNIQUE_ID_BYTES, "unique id size");
  ncclUniqueId u;
  RCCLCHK(ncclGetUniqueId(&u));
  memset(id, 0, MOX_UNIQUE_ID_BYTES);
  memcpy(id, &u, sizeof u);
  return MOX_OK;
}

int mox_comm_init(mox_engine* e, int nranks, int rank, const uint8_t id[MOX_UNIQUE_ID_BYTES]) {
  if (e && e->grp) return fail(MOX_EINVAL, "an engine group exchanges inside its own calls");
  if (!e || !id || nranks < 1 || rank < 0 || rank >= nranks) return fail(MOX_EINVAL, "bad communicator arguments");
  HIPCHK(hipSetDevice(e->device));
  if (e->comm) { ncclCommDestroy(e->comm); e->comm = nullptr; }
  ncclUniqueId u;
  memcpy(&u, id, sizeof u);
  RCCLCHK(ncclCommInitRank(&e->comm, nranks, u, rank));
  e->nranks = nranks;
  e->rank = rank;
  return MOX_OK;
}

int mox_run_shards(mox_engine* e, const mox_shard* shards) {
  if (!e || !shards) return fail(MOX_EINVAL, "NULL argument");
  if (!e->grp) {
    const mox_shard& s = shards[0];
    return mox_run_range(e, s.d_buf, s.buf_len, s.own_begin, s.own_end, s.at_corpus_end);
  }
  return group_run_shards(e, shards);
}

int mox_group_size(const mox_engine* e) { return e && e->grp ? e->grp->n : 1; }

mox_engine* mox_group_member(mox_engine* e, int i) {
  if (!e) return nullptr;
  if (!e->grp) return i == 0 ? e : nullptr;
  return i >= 0 && i < e->grp->n ? e->grp->m[i] : nullptr;
}

int mox_exchange(mox_engine* e) {
  if (!e) return fail(MOX_EINVAL, "engine is NULL");
  if (!e->comm) return fail(MOX_ESTATE, "mox_comm_init first");
  RcclTransport t(e);
  return exchange_impl(e, e->nranks, e->rank, t);
}

int mox_exchange_host(mox_engine* e, int nranks, int rank, mox_alltoallv_fn fn, void* user) {
  if (e && e->grp) return fail(MOX_EINVAL, "an engine group exchanges inside its own calls");
  if (!e || !fn) return fail(MOX_EINVAL, "NULL argument");
  if (nranks < 1 || nranks > MAX_RANKS || rank < 0 || rank >= nranks) return fail(MOX_EINVAL, "bad rank %d of %d", rank, nranks);
  HostTransport t(e, nranks, fn, user);
  return exchange_impl(e, nranks, rank, t);
}

int mox_gather(mox_engine* e, int root) {
  if (!e) return fail(MOX_EINVAL, "engine is NULL");
  if (!e->comm) return fail(MOX_ESTATE, "mox_comm_init first");
  RcclTransport t(e);
  return gather_impl(e, e->nranks, e->rank, root, t);
}

int mox_gather_host(mox_engine* e, int nranks, int rank, int root, mox_alltoallv_fn fn, void* user) {
  if (e && e->grp) return fail(MOX_EINVAL, "an engine group exchanges inside its own calls");
  if (!e || !fn) return fail(MOX_EINVAL, "NULL argument");
  if (nranks < 1 || nranks > MAX_RANKS || rank < 0 || rank >= nranks) return fail(MOX_EINVAL, "bad rank %d of %d", rank, nranks);
  HostTransport t(e, nranks, fn, user);
  return gather_impl(e, nranks, rank, root, t);
}

int mox_reduce_pairs(mox_engine* e, const uint8_t* bytes, const uint64_t* offs, const uint64_t* counts, uint64_t n) {
  if (!e || (n && (!bytes || !offs || !counts))) return fail(MOX_EINVAL, "NULL argument");
  return reduce_pairs_impl(e, bytes, offs, counts, n);
}

int mox_debug_exchange_layout(int nranks, const uint64_t* counts, uint64_t* out) {
  if (!counts || !out) return fail(MOX_EINVAL, "NULL argument");
  if (nranks < 1 || nranks > MAX_RANKS) return fail(MOX_EINVAL, "bad rank count %d", nranks);
  const int P = nranks;
  std::vector<XCnt> rows(2 * (size_t)P * P);
  std::vector<XCnt*> snd(P), rcv(P);
  for (int i = 0; i < P; i++) {
    snd[i] = rows.data() + (size_t)i * P;
    rcv[i] = rows.data() + (size_t)(P + i) * P;
    for (int d = 0; d < P; d++) {
      const uint64_t* c = counts + ((size_t)i * P + d) * 3;
      snd[i][d] = XCnt{c[0], c[1], c[2], 0};
    }
  }
  count_transpose(P, snd.data(), rcv.data());
  for (int i = 0; i < P; i++) {
    XPlan x;
    x.P = P;
    x_layout(x, snd[i], rcv[i]);
    const uint64_t* cols[8] = {x.s_short_off, x.s_short_len, x.s_blob_off, x.s_blob_len,
                               x.r_short_off, x.r_short_len, x.r_blob_off, x.r_blob_len};
    for (int k = 0; k < 8; k++)
      for (int d = 0; d < P; d++) out[((size_t)i * 8 + k) * P + d] = cols[k][d];
  }
  return MOX_OK;
}

}  // extern "C"

