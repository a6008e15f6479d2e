/* mox.h -- C ABI of the MI355X word-count engine (drop-in for the hot path of
 * AnarchistHoneybun/map-oxidize).
 *
 * The reference has no plugin / FFI API: the whole hot path is the private call
 * sequence in `main` (/root/reference/src/main.rs:16-22)
 *
 *     let chunks       = split_file("shakes.txt", 8).await?;                 // :16, fn :36-51
 *     let map_results  = map_phase(&chunks, 8).await?;                      // :19, fn :53-92
 *     let final_result = reduce_phase(map_results.clone(), 4).await?;       // :22, fn :111-150
 *
 * i.e. `path -> HashMap<String, usize>` consumed by write_final_result
 * (:170-182) and print_top_words (:184-192).  mox_count_file / mox_count
 * replace those three lines with one call that returns the same word -> count
 * table; mox_write_final_result / mox_print_top_words reproduce the L5 output.
 * INTEGRATION.md shows the Rust FFI binding a maintainer would add.
 *
 * Semantics (bit-exact with the reference): tokens are Rust
 * `str::split_whitespace` (Unicode White_Space delimiters) of the UTF-8 text,
 * each lowercased with Rust `str::to_lowercase` (full mapping + Final_Sigma),
 * counted with u64.  Invalid UTF-8 returns MOX_EUTF8 and no table, like the
 * reference's InvalidData abort at main.rs:44 -> :16.
 *
 * Conventions: every entry point returns an int status (0 = MOX_OK); no
 * exception crosses the ABI; mox_last_error() holds a thread-local message.
 * An engine is bound to one HIP device -- or, as an engine group
 * (mox_config.n_gpus > 1), drives several from the calling thread -- and is
 * not thread-safe (one host thread per engine).  Every call except mox_run_range_async is synchronous: it
 * returns after its work (and any pending asynchronous pass) is complete.
 * mox_run_range_async returns once its pass is queued; see its comment for
 * the lifetime rule of the device buffer it reads.
 */
#ifndef MOX_H
#define MOX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MOX_ABI_VERSION 4

/* status codes */
#define MOX_OK 0
#define MOX_EINVAL (-1)  /* bad argument */
#define MOX_EUTF8 (-2)   /* input is not valid UTF-8 (reference: io::ErrorKind::InvalidData) */
#define MOX_ENOMEM (-3)  /* device or host allocation failed */
#define MOX_EHIP (-4)    /* HIP runtime error */
#define MOX_EIO (-5)     /* file I/O error (reference: io::Error from File::open / reads) */
#define MOX_ERCCL (-6)   /* RCCL error */
#define MOX_ESTATE (-7)  /* call out of order (e.g. fetch before run) */
#define MOX_EHALO (-8)   /* a shard's token ran past the end of its buffer: halo too small */

/* mox_config.flags */
#define MOX_F_NO_DICT 0x1u      /* disable the hot-word dictionary (all tokens take the cold path) */
#define MOX_F_SORT_BYTES 0x2u   /* the result table is sorted bytewise ascending (Rust String Ord) on the GPU
                                   (at mox_fetch_table; an engine group: right after its gather, inside the
                                   mox_count / mox_run_shards call) instead of engine order */
#define MOX_F_TIMING 0x4u       /* record per-kernel HIP-event timings into mox_stats */
#define MOX_F_TIMING_MAP 0x8u   /* HIP events around the map kernel only (ms_map): each event record idles
                                   the stream ~5.6 us, so timed loops bracket just the dominant kernel */

#define MOX_MAX_GPUS 16
/* mox_config.transport of an engine group */
#define MOX_XPORT_RCCL 0u  /* RCCL communicators (ncclCommInitAll) over xGMI, one ncclGroupStart/End per all-to-all */
#define MOX_XPORT_COPY 1u  /* device-to-device copies (hipMemcpyPeerAsync); members may share a GPU (tests) */

typedef struct mox_config {
  int device;             /* HIP device ordinal; -1 = current device */
  uint32_t flags;         /* MOX_F_* */
  uint32_t dict_words;    /* hot dictionary capacity; 0 = default (4096, also the maximum) */
  uint32_t sample_pieces; /* 4 KiB pieces sampled to build the dictionary; 0 = default (192), max 1024 */
  uint64_t reserve_bytes; /* pre-size device buffers for corpora of this size (per GPU); 0 = grow on demand */
  /* engine group: n_gpus > 1 makes ONE engine that
     drives n_gpus GPUs from the calling thread.  mox_count / mox_count_file
     split the input into byte ranges at whitespace, run the local passes on
     all GPUs at once, exchange the partial tables (hash-partitioned
     all-to-all), reduce per owner and gather the final table on member 0;
     mox_run_shards does the same over device-resident shards. */
  uint32_t n_gpus;        /* 0 or 1: a single-GPU engine on `device` */
  uint32_t transport;     /* MOX_XPORT_* (engine group) */
  uint32_t n_devices;     /* 0: member i runs on device i; else n_gpus: member i runs on devices[i] */
  int32_t devices[MOX_MAX_GPUS];
  uint32_t reserved[5];
} mox_config;

typedef struct mox_engine mox_engine;

/* One shard of a device-resident corpus for mox_run_shards: the buffer lives
 * on the member's GPU; tokens whose first byte lies in [own_begin, own_end)
 * belong to it (see mox_run_range for the context / look-ahead rules). */
typedef struct mox_shard {
  const void* d_buf;
  size_t buf_len, own_begin, own_end;
  int at_corpus_end;
} mox_shard;

/* Result table: one entry per distinct lowercased word.  Engine order: words
 * of at most 16 bytes without a NUL byte first, ascending by (32-bit key hash,
 * second 32-bit key hash, the word's 16-byte zero-padded key) -- the same
 * whichever reduce kernel grouped the word -- then longer words in long-table
 * slot order (which can vary from run to run when two long words race for a
 * slot).  With
 * MOX_F_SORT_BYTES (or after mox_table_sort_bytes): bytewise ascending, Rust
 * String Ord, sorted on the GPU).  The reference's own order is HashMap-random
 * (/root/reference/src/main.rs:177-179).  After mox_gather the root's table
 * is the ranks' tables one after another (rank order), each in engine order;
 * an engine group's gathered table likewise, unless MOX_F_SORT_BYTES.
 * Memory is owned by the library until mox_table_free. */
typedef struct mox_table {
  uint64_t n;              /* distinct words */
  uint64_t tokens;         /* total tokens counted (== sum of counts) */
  const uint64_t* counts;  /* [n] */
  const uint64_t* offs;    /* [n+1] byte offsets into bytes */
  const uint8_t* bytes;    /* concatenated UTF-8 words */
} mox_table;

typedef struct mox_stats {
  uint64_t bytes;          /* corpus bytes of the last run */
  uint64_t tokens;
  uint64_t uniques;
  uint64_t dict_words;     /* words in the hot dictionary */
  uint64_t cold_records;   /* tokens that took the cold (partitioned) path */
  uint64_t weighted_records;
  uint64_t unicode_tokens; /* tokens that went through the Unicode case lane */
  uint64_t long_tokens;    /* tokens longer than 16 bytes (hashed keys + byte compare) */
  uint64_t chunks;         /* cold-record chunks allocated */
  uint32_t retries;        /* buffer-growth reruns in the last call */
  uint32_t max_subpasses;  /* largest reduce sub-pass count of any bucket */
  /* device milliseconds (HIP events on the engine stream; MOX_F_TIMING) */
  double ms_run;           /* whole device pipeline: corpus in HBM -> table in HBM */
  double ms_dict;          /* sample + dictionary build */
  double ms_map;           /* map kernel (dominant kernel) */
  double ms_lanes;         /* unicode + long lanes */
  double ms_reduce;        /* directory + bucket reduce */
  double ms_finalize;      /* table materialisation */
  double ms_h2d;           /* host -> device corpus copy (mox_count / mox_count_file) */
  double ms_d2h;           /* table fetch */
  double ms_exchange;      /* multi-GPU all-to-all + final reduce (not the sorted exchange's sort: ms_sort) */
  uint64_t reduce_units;   /* reduce work units (partitions, or their sub-buckets when split) */
  uint32_t split_partitions; /* partitions split by the high-cardinality path */
  uint32_t async_reruns;   /* async passes re-run synchronously (overflow), cumulative over the engine */
  /* multi-GPU (last mox_exchange / mox_gather of this rank) */
  uint64_t x_bytes_sent;   /* exchange payload bytes this rank sent (records + long-word blobs, self included) */
  uint64_t x_bytes_recv;   /* exchange payload bytes this rank received */
  uint64_t gather_bytes;   /* table bytes this rank sent to the gather root (root: received) */
  double ms_gather;        /* wall time of the last mox_gather on this rank */
  /* exactness-fallback hit counters of the last pass (a local pass plus its
     exchange's reduce pass), counted only by the forced-collision check build
     (libmox_hc.so, -DMOX_HASH_COLLIDE); zero in production builds:
     [0] dictionary tag equal, key different   [1] long-word table: equal hash, different bytes
     [2] one-wave sort reduce re-sorted on 64-bit keys   [3] ... handed its unit to k_reduce
     [4] k_reduce table: equal tag, different key   [5] k_reduce_small: equal hash, different key */
  uint64_t path_hits[8];
  double ms_sort;          /* device bytewise table sort (MOX_F_SORT_BYTES), wall time */
  double ms_local;         /* engine group: local passes of all members (wall time) */
  uint32_t n_gpus;         /* engine group size (1 for a single-GPU engine) */
  uint32_t async_dropped;  /* overflowed async passes superseded by a later queued pass (never re-run) */
  uint32_t x_ranged;       /* the last exchange owned words by byte range (MOX_F_SORT_BYTES); 0: by hash
                              (no sort flag, or skewed 8-byte prefixes fell back to hash owners) */
  uint32_t x_pad;
} mox_stats;

const char* mox_last_error(void);
int mox_abi_version(void);

int mox_engine_create(const mox_config* cfg, mox_engine** out);
/* Replace the engine's MOX_F_* flags (e.g. switch timing modes between runs); an
 * engine group applies them to every member. */
int mox_set_flags(mox_engine* e, uint32_t flags);
void mox_engine_destroy(mox_engine* e);

/* ---- drop-in for main.rs:16-22 ---- */
/* Count words of a host buffer (copied to HBM first). */
int mox_count(mox_engine* e, const uint8_t* text, size_t len, mox_table** out);
/* Count words of a file (reference: split_file(path) .. reduce_phase). */
int mox_count_file(mox_engine* e, const char* path, mox_table** out);
void mox_table_free(mox_table* t);
/* Reorder a fetched table bytewise ascending (Rust String Ord) in place. */
int mox_table_sort_bytes(mox_table* t);

/* ---- device-resident path (bench / pipelines): corpus already in HBM ---- */
/* One full pass: HBM corpus -> HBM table.  No host copy of the result. */
int mox_run_device(mox_engine* e, const void* d_text, size_t len);
/* Same over a shard window: count tokens whose first byte lies in
 * [own_begin, own_end) of the buffer d_buf[0, buf_len).  Bytes before own_begin
 * give the left context (own_begin == 0 means "corpus start"); bytes after
 * own_end are look-ahead for the last token.  at_corpus_end != 0 means the
 * buffer end is the end of the corpus; otherwise a token reaching the buffer
 * end is an error (MOX_EHALO). */
int mox_run_range(mox_engine* e, const void* d_buf, size_t buf_len, size_t own_begin, size_t own_end,
                  int at_corpus_end);
/* Asynchronous mox_run_range: enqueues the pass and returns; the pass queued
 * by the previous async call is completed (checked, and re-run synchronously
 * if a buffer overflowed) after this one is enqueued, so back-to-back passes
 * leave no host round trip between them on the GPU.  A pass's error is
 * returned by the call that completes it: the next mox_run_range_async, or
 * mox_run_wait.  Every other entry point completes pending passes first.
 * Buffer lifetime: an overflowed pass is re-run later from d_buf, so d_buf
 * must stay valid and unmodified until the call that completes the pass has
 * returned (the next mox_run_range_async, mox_run_wait, or any other entry
 * point of this engine).  An overflowed pass with a later pass already queued
 * behind it is not re-run: the later pass supersedes its table
 * (mox_stats.async_dropped). */
int mox_run_range_async(mox_engine* e, const void* d_buf, size_t buf_len, size_t own_begin, size_t own_end,
                        int at_corpus_end);
/* Complete every pending async pass; the last one's table is the result. */
int mox_run_wait(mox_engine* e);
/* Engine group: one call for n_gpus device-resident shards (shards[i] on
 * member i's GPU): local passes on every GPU at once, exchange, final
 * reduce, gather on member 0 (and the bytewise sort with MOX_F_SORT_BYTES).
 * A single-GPU engine takes one shard (= mox_run_range). */
int mox_run_shards(mox_engine* e, const mox_shard* shards);
/* Members of an engine group (1 for a single-GPU engine); member 0 is e
 * itself.  A member's engine serves device allocations and copies for its
 * shard (mox_device_alloc / mox_memcpy_h2d). */
int mox_group_size(const mox_engine* e);
mox_engine* mox_group_member(mox_engine* e, int i);
/* Copy the table of the last run (or of the last exchange) to the host. */
int mox_fetch_table(mox_engine* e, mox_table** out);
/* Reorder the device-resident result table bytewise ascending (Rust String
 * Ord) on the GPU, without fetching it (e.g. the root's table after
 * mox_gather, inside a timed multi-GPU step).  MOX_ENOMEM when the sort's
 * device scratch cannot be allocated: the table then stays in engine order
 * (mox_fetch_table with MOX_F_SORT_BYTES still sorts it, on the host). */
int mox_sort_result(mox_engine* e);
int mox_get_stats(const mox_engine* e, mox_stats* out);

/* device memory helpers so callers need no HIP headers */
int mox_device_alloc(mox_engine* e, size_t bytes, void** d_ptr);
int mox_device_free(mox_engine* e, void* d_ptr);
int mox_memcpy_h2d(mox_engine* e, void* d_dst, const void* h_src, size_t bytes);
int mox_memcpy_d2h(mox_engine* e, void* h_dst, const void* d_src, size_t bytes);
int mox_synchronize(mox_engine* e);

/* ---- multi-GPU (one process per GPU, RCCL over xGMI) ---- */
#define MOX_UNIQUE_ID_BYTES 128
int mox_comm_unique_id(uint8_t id[MOX_UNIQUE_ID_BYTES]);
int mox_comm_init(mox_engine* e, int nranks, int rank, const uint8_t id[MOX_UNIQUE_ID_BYTES]);
/* After mox_run_range on every rank: hash-partition the local table, exchange
 * it with one RCCL all-to-all, and reduce the received partials.  Afterwards
 * this rank owns the final counts of its hash range (disjoint across ranks).
 * With MOX_F_SORT_BYTES the words are owned by byte range instead (splitters
 * from 1,024 sampled 8-byte prefixes per rank, exchanged first) and every rank
 * sorts its own range on its GPU, so mox_gather in rank order is the table in
 * bytewise order (no sort at the root). */
int mox_exchange(mox_engine* e);
/* Host-staged transport for the same exchange (several ranks sharing one GPU,
 * or no RCCL): the library calls fn once per all-to-all with pinned host
 * buffers; send holds nranks consecutive blocks of send_bytes[d] bytes for
 * rank d, recv must receive nranks consecutive blocks of recv_bytes[s] bytes
 * from rank s.  Return 0 on success. */
typedef int (*mox_alltoallv_fn)(void* user, const void* send, const uint64_t* send_bytes, void* recv,
                                const uint64_t* recv_bytes);
int mox_exchange_host(mox_engine* e, int nranks, int rank, mox_alltoallv_fn fn, void* user);
/* After mox_exchange on every rank: gather the ranks' final tables into the
 * root's engine (RCCL send/recv, device to device).  Ranks own disjoint words
 * after the exchange, so the root's table afterwards is the whole corpus's
 * table (fetch it with mox_fetch_table; MOX_F_SORT_BYTES gives bytewise order).
 * Other ranks keep their own table.  Replaces the reference's single-process
 * result (main.rs:22) for one process per GPU. */
int mox_gather(mox_engine* e, int root);
/* The same over the host-staged transport of mox_exchange_host. */
int mox_gather_host(mox_engine* e, int nranks, int rank, int root, mox_alltoallv_fn fn, void* user);

/* ---- output layer (reference L5: main.rs:170-192) ---- */
/* final_result.txt: one "{word} {count}\n" line per word.  Truncates on open
 * (the reference does not: SURVEY.md §0.2 quirk, not reproduced). */
int mox_write_final_result(const mox_table* t, const char* path);
/* "Top {n} words:" then up to n lines "{word}: {count}", count descending,
 * ties in table order (the reference's tie order is HashMap-random). */
int mox_print_top_words(const mox_table* t, size_t n);

/* ---- intermediate (spill) files, SURVEY.md §8(f) rank 4 ---- */
/* reduce_phase over parsed map files (replaces main.rs:111-150; the parse of
 * read_map_result main.rs:152-168 is host text work): n (word, count) pairs,
 * word i = bytes[offs[i], offs[i+1]) taken verbatim (not lowercased), are
 * summed by word with the GPU reduce; the result is then fetched with
 * mox_fetch_table like a run's.  Duplicate words are summed. */
int mox_reduce_pairs(mox_engine* e, const uint8_t* bytes, const uint64_t* offs, const uint64_t* counts, uint64_t n);

/* ---- test hook (no GPU needed) ---- */
/* The exchange's per-peer send / receive layout (mox_multi.hip x_layout) for
 * nranks ranks whose count rows are counts[i][d][0..2] = (short records, long
 * words, long-word bytes) that rank i sends to rank d, the count all-to-all
 * modelled as the device-copy transport does it.  out[i][k][d], k = 0..7:
 * short send offset / length, blob send offset / length, short receive offset /
 * length, blob receive offset / length of rank i for peer d (bytes). */
int mox_debug_exchange_layout(int nranks, const uint64_t* counts, uint64_t* out);

#ifdef __cplusplus
}
#endif
#endif /* MOX_H */
