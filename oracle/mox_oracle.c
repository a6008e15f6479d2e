/* ORACLE -- test infrastructure only.  Never linked into, loaded by, or called
 * from the product path (map-oxidize_amd/).  Only tests/, __graft_entry__.smoke()
 * and bench.py's cpu_baseline leg may use it, and only as the checker.
 *
 * CPU restatement of the reference's word count (AnarchistHoneybun/map-oxidize,
 * /root/reference/src/main.rs):
 *   - UTF-8 validity: tokio `lines()` rejects invalid UTF-8 (InvalidData), which
 *     aborts `split_file` via `?` (main.rs:44) and `main` (main.rs:16) before any
 *     output.  A file is valid line-by-line iff it is valid as a whole (0x0A never
 *     occurs inside a multi-byte sequence), so the whole buffer is validated.
 *   - tokens: `text.split_whitespace()` (main.rs:96) = maximal runs of chars that
 *     are not Unicode White_Space (Rust `char::is_whitespace`).
 *   - case: `word.to_lowercase()` (main.rs:97) = per-char full lowercase mapping
 *     plus the Final_Sigma rule (Rust core `str::to_lowercase`/`map_uppercase_sigma`).
 *   - counts: `*word_counts.entry(word).or_insert(0) += 1` (main.rs:98), then the
 *     per-chunk maps are summed (main.rs:132-134).  The round-robin line chunking
 *     (main.rs:41-48) splits only at '\n', which is whitespace, so the sum equals
 *     one global count over the whole text.  Counts are usize (u64).
 *   - output: the reference writes HashMap order (random, main.rs:177-179); the
 *     oracle returns entries sorted bytewise (Rust String Ord) for comparison.
 *
 * PARITY UNPINNED: the reference is Rust, no Rust toolchain exists in this image
 * and the reference ships no tests, fixtures or golden outputs (SURVEY.md §4,
 * §8(c)).  This restatement is cross-checked against an independent Python
 * restatement (oracle/pyoracle.py: Python's strict UTF-8 decoder, an explicit
 * White_Space set and str.lower()) and the known-answer table of SURVEY.md §0.1.
 * Case data: Unicode 14.0.0 from ICU 70.1, in the oracle's own tables
 * (oracle/mox_oracle_case.h, written by oracle/gen_case_tables.py from the ICU
 * fixture tests/golden/unicode_icu70.json); neither the product's table header
 * nor its lookup code is used here.  tests/test_unicode_pin.py pins the
 * product header, and this oracle, to the same ICU answers (lowercase map,
 * Final_Sigma probes, White_Space).
 */
#include "mox_oracle.h"

#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#include "mox_oracle_case.h" /* the oracle's own tables, from the ICU 70.1 fixture (gen_case_tables.py) */

/* ---- UTF-8 validation (Rust core::str::from_utf8 rules) ---- */
int64_t moxo_utf8_invalid_at(const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  while (i < n) {
    uint8_t c = s[i];
    if (c < 0x80) { i++; continue; }
    uint32_t need;
    uint8_t lo = 0x80, hi = 0xBF;
    if (c >= 0xC2 && c <= 0xDF) need = 1;
    else if (c == 0xE0) { need = 2; lo = 0xA0; }
    else if (c >= 0xE1 && c <= 0xEC) need = 2;
    else if (c == 0xED) { need = 2; hi = 0x9F; }
    else if (c >= 0xEE && c <= 0xEF) need = 2;
    else if (c == 0xF0) { need = 3; lo = 0x90; }
    else if (c >= 0xF1 && c <= 0xF3) need = 3;
    else if (c == 0xF4) { need = 3; hi = 0x8F; }
    else return (int64_t)i;
    if (i + need >= n) return (int64_t)i; /* truncated sequence at the end */
    if (s[i + 1] < lo || s[i + 1] > hi) return (int64_t)i;
    for (uint32_t k = 2; k <= need; k++)
      if ((s[i + k] & 0xC0) != 0x80) return (int64_t)i;
    i += need + 1;
  }
  return -1;
}

static inline uint32_t dec(const uint8_t* s, uint64_t* i) { /* valid input only */
  uint8_t c = s[*i];
  if (c < 0x80) { (*i)++; return c; }
  if (c < 0xE0) { uint32_t v = ((uint32_t)(c & 0x1F) << 6) | (s[*i + 1] & 0x3F); *i += 2; return v; }
  if (c < 0xF0) {
    uint32_t v = ((uint32_t)(c & 0x0F) << 12) | ((uint32_t)(s[*i + 1] & 0x3F) << 6) | (s[*i + 2] & 0x3F);
    *i += 3; return v;
  }
  uint32_t v = ((uint32_t)(c & 0x07) << 18) | ((uint32_t)(s[*i + 1] & 0x3F) << 12) |
               ((uint32_t)(s[*i + 2] & 0x3F) << 6) | (s[*i + 3] & 0x3F);
  *i += 4; return v;
}

static inline int enc(uint32_t cp, uint8_t* o) {
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

/* Rust char::is_whitespace == Unicode White_Space */
int moxo_is_whitespace(uint32_t c) {
  if (c <= 0x7F) return c == 0x20 || (c >= 0x09 && c <= 0x0D);
  switch (c) {
    case 0x85: case 0xA0: case 0x1680: case 0x2028: case 0x2029: case 0x202F: case 0x205F: case 0x3000: return 1;
    default: return c >= 0x2000 && c <= 0x200A;
  }
}

static int in_ranges(uint32_t c, const moxo_range_t* r, int n) {
  int a = 0, b = n - 1;
  while (a <= b) {
    int m = (a + b) >> 1;
    if (c < r[m].lo) b = m - 1;
    else if (c > r[m].hi) a = m + 1;
    else return 1;
  }
  return 0;
}
static int is_cased(uint32_t c) { return in_ranges(c, moxo_cased, MOXO_CASED_N); }
static int is_ci(uint32_t c) { return in_ranges(c, moxo_ci, MOXO_CI_N); }
/* lowercase of c: one or two code points (*second = 0: one) */
static uint32_t lower1(uint32_t c, uint32_t* second) {
  int a = 0, b = MOXO_LOWER_N - 1;
  *second = 0;
  while (a <= b) {
    int m = (a + b) >> 1;
    if (c < moxo_lower[m].cp) b = m - 1;
    else if (c > moxo_lower[m].cp) a = m + 1;
    else {
      *second = moxo_lower[m].l1;
      return moxo_lower[m].l0;
    }
  }
  return c;
}

/* Lowercase token s[0..n) (valid UTF-8) into out (capacity >= 3*n/2+4).  Returns length. */
uint64_t moxo_lowercase(const uint8_t* s, uint64_t n, uint8_t* out) {
  int ascii = 1;
  for (uint64_t i = 0; i < n; i++) if (s[i] >= 0x80) { ascii = 0; break; }
  if (ascii) {
    for (uint64_t i = 0; i < n; i++) out[i] = (s[i] >= 'A' && s[i] <= 'Z') ? (uint8_t)(s[i] + 32) : s[i];
    return n;
  }
  /* decode to code points */
  uint32_t* cps = (uint32_t*)malloc((n + 1) * sizeof(uint32_t));
  uint64_t m = 0, i = 0, o = 0;
  while (i < n) cps[m++] = dec(s, &i);
  for (uint64_t k = 0; k < m; k++) {
    uint32_t c = cps[k];
    if (c == 0x3A3) {
      /* Final_Sigma: cased (after skipping case-ignorable) before, and not
       * (case-ignorable* cased) after -- Rust map_uppercase_sigma. */
      int64_t j = (int64_t)k - 1;
      while (j >= 0 && is_ci(cps[j])) j--;
      int fin = j >= 0 && is_cased(cps[j]);
      if (fin) {
        uint64_t q = k + 1;
        while (q < m && is_ci(cps[q])) q++;
        if (q < m && is_cased(cps[q])) fin = 0;
      }
      o += (uint64_t)enc(fin ? 0x3C2 : 0x3C3, out + o);
      continue;
    }
    uint32_t l2;
    const uint32_t l = lower1(c, &l2);
    o += (uint64_t)enc(l, out + o);
    if (l2) o += (uint64_t)enc(l2, out + o);
  }
  free(cps);
  return o;
}

/* ---- counting hash map ---- */
typedef struct { uint64_t h, off, len, count; } slot_t;
typedef struct {
  slot_t* slots; uint64_t cap, n;
  uint8_t* arena; uint64_t alen, acap;
  uint64_t tokens;
} cmap;

static uint64_t fnv(const uint8_t* s, uint64_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < n; i++) { h ^= s[i]; h *= 0x100000001b3ull; }
  return h | 1;
}
static void cmap_init(cmap* m) {
  m->cap = 1024; m->n = 0; m->slots = (slot_t*)calloc(m->cap, sizeof(slot_t));
  m->acap = 1 << 16; m->alen = 0; m->arena = (uint8_t*)malloc(m->acap); m->tokens = 0;
}
static void cmap_grow(cmap* m) {
  uint64_t nc = m->cap * 2;
  slot_t* ns = (slot_t*)calloc(nc, sizeof(slot_t));
  for (uint64_t i = 0; i < m->cap; i++) if (m->slots[i].h) {
    uint64_t j = m->slots[i].h & (nc - 1);
    while (ns[j].h) j = (j + 1) & (nc - 1);
    ns[j] = m->slots[i];
  }
  free(m->slots); m->slots = ns; m->cap = nc;
}
static void cmap_add(cmap* m, const uint8_t* w, uint64_t len, uint64_t cnt) {
  uint64_t h = fnv(w, len), j = h & (m->cap - 1);
  for (;;) {
    slot_t* s = &m->slots[j];
    if (!s->h) break;
    if (s->h == h && s->len == len && memcmp(m->arena + s->off, w, len) == 0) { s->count += cnt; return; }
    j = (j + 1) & (m->cap - 1);
  }
  if (m->alen + len > m->acap) {
    while (m->alen + len > m->acap) m->acap *= 2;
    m->arena = (uint8_t*)realloc(m->arena, m->acap);
  }
  memcpy(m->arena + m->alen, w, len);
  m->slots[j] = (slot_t){h, m->alen, len, cnt};
  m->alen += len; m->n++;
  if (m->n * 2 > m->cap) cmap_grow(m);
}
static void cmap_free(cmap* m) { free(m->slots); free(m->arena); }

/* count_words (main.rs:94-101) over s[0..n), valid UTF-8 */
static void count_range(cmap* m, const uint8_t* s, uint64_t n) {
  uint64_t i = 0;
  uint8_t* buf = NULL;
  uint64_t bcap = 0;
  while (i < n) {
    uint64_t p = i;
    uint32_t c = dec(s, &p);
    if (moxo_is_whitespace(c)) { i = p; continue; }
    uint64_t start = i;
    i = p;
    while (i < n) {
      uint64_t q = i;
      uint32_t d = dec(s, &q);
      if (moxo_is_whitespace(d)) break;
      i = q;
    }
    uint64_t len = i - start;
    if (len * 2 + 8 > bcap) { bcap = len * 2 + 8; buf = (uint8_t*)realloc(buf, bcap); }
    uint64_t ll = moxo_lowercase(s + start, len, buf);
    cmap_add(m, buf, ll, 1);
    m->tokens++;
  }
  free(buf);
}

typedef struct { cmap m; const uint8_t* s; uint64_t n; } tjob;
static void* tmain(void* a) { tjob* j = (tjob*)a; count_range(&j->m, j->s, j->n); return NULL; }

static const uint8_t* g_sort_arena;
static const slot_t* g_sort_slots;
static int cmp_idx(const void* a, const void* b) {
  const slot_t* x = &g_sort_slots[*(const uint64_t*)a];
  const slot_t* y = &g_sort_slots[*(const uint64_t*)b];
  uint64_t l = x->len < y->len ? x->len : y->len;
  int c = memcmp(g_sort_arena + x->off, g_sort_arena + y->off, l);
  if (c) return c;
  return x->len < y->len ? -1 : x->len > y->len ? 1 : 0;
}

int moxo_count(const uint8_t* s, uint64_t n, int nthreads, moxo_table* out) {
  memset(out, 0, sizeof(*out));
  int64_t bad = moxo_utf8_invalid_at(s, n);
  if (bad >= 0) { out->invalid_at = bad; return MOXO_EUTF8; }
  out->invalid_at = -1;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  /* split at '\n' (always whitespace), like the reference's line chunking */
  uint64_t cuts[65];
  int nt = 0;
  cuts[0] = 0;
  for (int t = 1; t < nthreads; t++) {
    uint64_t p = n / (uint64_t)nthreads * (uint64_t)t;
    if (p < cuts[nt]) p = cuts[nt];
    while (p < n && s[p] != '\n') p++;
    if (p < n && p > cuts[nt]) cuts[++nt] = p;
  }
  cuts[++nt] = n;
  tjob* jobs = (tjob*)calloc((size_t)nt, sizeof(tjob));
  pthread_t th[64];
  for (int t = 0; t < nt; t++) {
    cmap_init(&jobs[t].m);
    jobs[t].s = s + cuts[t]; jobs[t].n = cuts[t + 1] - cuts[t];
    if (nt > 1) pthread_create(&th[t], NULL, tmain, &jobs[t]); else tmain(&jobs[t]);
  }
  if (nt > 1) for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
  cmap* g = &jobs[0].m;
  for (int t = 1; t < nt; t++) {
    cmap* m = &jobs[t].m;
    for (uint64_t i = 0; i < m->cap; i++)
      if (m->slots[i].h) cmap_add(g, m->arena + m->slots[i].off, m->slots[i].len, m->slots[i].count);
    g->tokens += m->tokens;
    cmap_free(m);
  }
  uint64_t* idx = (uint64_t*)malloc((g->n + 1) * sizeof(uint64_t));
  uint64_t k = 0;
  for (uint64_t i = 0; i < g->cap; i++) if (g->slots[i].h) idx[k++] = i;
  g_sort_arena = g->arena; g_sort_slots = g->slots;
  qsort(idx, k, sizeof(uint64_t), cmp_idx);
  out->n = k;
  out->tokens = g->tokens;
  out->counts = (uint64_t*)malloc((k + 1) * sizeof(uint64_t));
  out->offs = (uint64_t*)malloc((k + 1) * sizeof(uint64_t));
  out->bytes = (uint8_t*)malloc(g->alen + 1);
  uint64_t o = 0;
  for (uint64_t i = 0; i < k; i++) {
    const slot_t* sl = &g->slots[idx[i]];
    out->offs[i] = o; out->counts[i] = sl->count;
    memcpy(out->bytes + o, g->arena + sl->off, sl->len);
    o += sl->len;
  }
  out->offs[k] = o;
  out->bytes_len = o;
  free(idx);
  cmap_free(g);
  free(jobs);
  return 0;
}

/* Tokens whose FIRST byte lies in [own_begin, own_end) of s[0, n) -- the shard
 * ownership rule of the multi-GPU split.  Bytes before
 * own_begin are left context (own_begin == 0: corpus start); bytes after own_end
 * are look-ahead; n is the corpus end.  Same table format as moxo_count. */
int moxo_count_range(const uint8_t* s, uint64_t n, uint64_t own_begin, uint64_t own_end, moxo_table* out) {
  memset(out, 0, sizeof(*out));
  int64_t bad = moxo_utf8_invalid_at(s, n);
  if (bad >= 0) { out->invalid_at = bad; return MOXO_EUTF8; }
  out->invalid_at = -1;
  /* start of the char containing own_begin */
  uint64_t p = own_begin;
  while (p > 0 && p < n && (s[p] & 0xC0) == 0x80) p--;
  int inside = 0; /* is p inside a token that started before own_begin? */
  if (p < own_begin) {
    uint64_t q = p;
    uint32_t c = dec(s, &q);
    if (!moxo_is_whitespace(c)) inside = 1;
    else p = q;
  } else if (p > 0 && p < n) {
    uint64_t b = p - 1;
    while (b > 0 && (s[b] & 0xC0) == 0x80) b--;
    uint64_t q = b;
    uint32_t c = dec(s, &q);
    if (!moxo_is_whitespace(c)) inside = 1;
  }
  if (inside) {
    while (p < n) {
      uint64_t q = p;
      uint32_t c = dec(s, &q);
      if (moxo_is_whitespace(c)) break;
      p = q;
    }
  }
  /* count tokens starting in [p, own_end) */
  cmap m;
  cmap_init(&m);
  uint8_t* buf = NULL;
  uint64_t bcap = 0;
  while (p < n) {
    uint64_t q = p;
    uint32_t c = dec(s, &q);
    if (moxo_is_whitespace(c)) { p = q; continue; }
    if (p >= own_end) break;
    uint64_t st = p;
    p = q;
    while (p < n) {
      uint64_t r = p;
      uint32_t d = dec(s, &r);
      if (moxo_is_whitespace(d)) break;
      p = r;
    }
    uint64_t len = p - st;
    if (len * 2 + 8 > bcap) { bcap = len * 2 + 8; buf = (uint8_t*)realloc(buf, bcap); }
    uint64_t ll = moxo_lowercase(s + st, len, buf);
    cmap_add(&m, buf, ll, 1);
    m.tokens++;
  }
  free(buf);
  uint64_t* idx = (uint64_t*)malloc((m.n + 1) * sizeof(uint64_t));
  uint64_t k = 0;
  for (uint64_t i = 0; i < m.cap; i++) if (m.slots[i].h) idx[k++] = i;
  g_sort_arena = m.arena; g_sort_slots = m.slots;
  qsort(idx, k, sizeof(uint64_t), cmp_idx);
  out->n = k; out->tokens = m.tokens;
  out->counts = (uint64_t*)malloc((k + 1) * sizeof(uint64_t));
  out->offs = (uint64_t*)malloc((k + 1) * sizeof(uint64_t));
  out->bytes = (uint8_t*)malloc(m.alen + 1);
  uint64_t o = 0;
  for (uint64_t i = 0; i < k; i++) {
    const slot_t* sl = &m.slots[idx[i]];
    out->offs[i] = o; out->counts[i] = sl->count;
    memcpy(out->bytes + o, m.arena + sl->off, sl->len);
    o += sl->len;
  }
  out->offs[k] = o; out->bytes_len = o;
  free(idx);
  cmap_free(&m);
  return 0;
}

void moxo_free(moxo_table* t) {
  free(t->counts); free(t->offs); free(t->bytes);
  memset(t, 0, sizeof(*t));
}

/* ---- property checks for corpora too large for a full sorted table ----
 * (tests/test_gpu_scale.py: C4 at >= 4 GiB, C4/C5 at 16 GiB).  Same
 * tokenizer, case folding and counting rules as moxo_count above. */

static uint64_t mix64(uint64_t x) { /* splitmix64 finaliser */
  x ^= x >> 30; x *= 0xbf58476d1ce4e5b9ull;
  x ^= x >> 27; x *= 0x94d049bb133111ebull;
  return x ^ (x >> 31);
}
static uint64_t fnv_full(const uint8_t* s, uint64_t n) {
  uint64_t h = 0xcbf29ce484222325ull;
  for (uint64_t i = 0; i < n; i++) { h ^= s[i]; h *= 0x100000001b3ull; }
  return h;
}
/* Order-independent digest of one (word, count) entry, summed over a table. */
static void digest_add(uint64_t d[4], const uint8_t* w, uint64_t len, uint64_t cnt) {
  const uint64_t x = mix64(fnv_full(w, len) ^ (cnt * 0x9E3779B97F4A7C15ull) ^ (len << 56));
  d[0] += 1; d[1] += cnt; d[2] += x; d[3] += mix64(x + 0x632BE59BD9B4E019ull);
}

/* Cuts of s[0, n) into at most nt pieces at '\n' bytes (cuts[0..nt]). */
static int cut_lines(const uint8_t* s, uint64_t n, int nthreads, uint64_t* cuts) {
  int nt = 0;
  cuts[0] = 0;
  for (int t = 1; t < nthreads; t++) {
    uint64_t p = n / (uint64_t)nthreads * (uint64_t)t;
    if (p < cuts[nt]) p = cuts[nt];
    while (p < n && s[p] != '\n') p++;
    if (p < n && p > cuts[nt]) cuts[++nt] = p;
  }
  cuts[++nt] = n;
  return nt;
}

/* Calls f(ctx, lowered word, len) for every token of s[0, n) (valid UTF-8). */
typedef void (*tok_fn)(void* ctx, const uint8_t* w, uint64_t len);
static uint64_t for_tokens(const uint8_t* s, uint64_t n, tok_fn f, void* ctx) {
  uint64_t i = 0, tokens = 0, bcap = 0;
  uint8_t* buf = NULL;
  while (i < n) {
    uint64_t p = i;
    uint32_t c = dec(s, &p);
    if (moxo_is_whitespace(c)) { i = p; continue; }
    uint64_t start = i;
    i = p;
    while (i < n) {
      uint64_t q = i;
      uint32_t d = dec(s, &q);
      if (moxo_is_whitespace(d)) break;
      i = q;
    }
    tokens++;
    if (!f) continue;
    uint64_t len = i - start;
    if (len * 2 + 8 > bcap) { bcap = len * 2 + 8; buf = (uint8_t*)realloc(buf, bcap); }
    f(ctx, buf, moxo_lowercase(s + start, len, buf));
  }
  free(buf);
  return tokens;
}

typedef struct { uint8_t* p; uint64_t n, cap; } bytevec;
static void bv_put(bytevec* v, const void* x, uint64_t k) {
  if (v->n + k > v->cap) {
    v->cap = v->cap ? v->cap * 2 : 1 << 20;
    while (v->n + k > v->cap) v->cap *= 2;
    v->p = (uint8_t*)realloc(v->p, v->cap);
  }
  memcpy(v->p + v->n, x, k);
  v->n += k;
}

typedef struct {
  const uint8_t* s; uint64_t n; int T; int t;
  bytevec* out;      /* [T] words routed to their owner thread: u32 len + bytes */
  uint64_t tokens;
  void* all;         /* the job array (phase 2 reads every job's out[t]) */
  uint64_t d[4];
} djob;
static void route(void* ctx, const uint8_t* w, uint64_t len) {
  djob* j = (djob*)ctx;
  const uint32_t owner = (uint32_t)(((fnv_full(w, len) >> 32) * (uint64_t)j->T) >> 32);
  const uint32_t l32 = (uint32_t)len;
  bv_put(&j->out[owner], &l32, 4);
  bv_put(&j->out[owner], w, len);
}
static void* dphase1(void* a) { djob* j = (djob*)a; j->tokens = for_tokens(j->s, j->n, route, j); return NULL; }
static void* dphase2(void* a) {
  djob* j = (djob*)a;
  djob* all = (djob*)j->all;
  cmap m;
  cmap_init(&m);
  for (int t = 0; t < j->T; t++) {
    bytevec* v = &all[t].out[j->t];
    for (uint64_t o = 0; o < v->n;) {
      uint32_t len;
      memcpy(&len, v->p + o, 4);
      cmap_add(&m, v->p + o + 4, len, 1);
      o += 4 + len;
    }
  }
  memset(j->d, 0, sizeof j->d);
  for (uint64_t i = 0; i < m.cap; i++)
    if (m.slots[i].h) digest_add(j->d, m.arena + m.slots[i].off, m.slots[i].len, m.slots[i].count);
  cmap_free(&m);
  return NULL;
}

/* Digest {distinct words, total count, sum1, sum2} of the word count of
 * s[0, n), without building the sorted table: tokens are routed to T owner
 * threads by hash, each owner counts its words.  Returns MOXO_EUTF8 on invalid
 * input, else 0; out[4] = digest, *tokens = token count. */
int moxo_count_digest(const uint8_t* s, uint64_t n, int nthreads, uint64_t out[4], uint64_t* tokens) {
  memset(out, 0, 4 * sizeof(uint64_t));
  *tokens = 0;
  if (moxo_utf8_invalid_at(s, n) >= 0) return MOXO_EUTF8;
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  uint64_t cuts[65];
  const int nt = cut_lines(s, n, nthreads, cuts);
  djob* jobs = (djob*)calloc((size_t)nt, sizeof(djob));
  pthread_t th[64];
  for (int t = 0; t < nt; t++) {
    jobs[t] = (djob){s + cuts[t], cuts[t + 1] - cuts[t], nt, t, (bytevec*)calloc((size_t)nt, sizeof(bytevec)), 0, jobs, {0, 0, 0, 0}};
    pthread_create(&th[t], NULL, dphase1, &jobs[t]);
  }
  for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
  for (int t = 0; t < nt; t++) pthread_create(&th[t], NULL, dphase2, &jobs[t]);
  for (int t = 0; t < nt; t++) pthread_join(th[t], NULL);
  for (int t = 0; t < nt; t++) {
    for (int k = 0; k < 4; k++) out[k] += jobs[t].d[k];
    *tokens += jobs[t].tokens;
    for (int d = 0; d < nt; d++) free(jobs[t].out[d].p);
    free(jobs[t].out);
  }
  free(jobs);
  return 0;
}

/* The same digest of a table (counts[n], offs[n+1], bytes), e.g. the GPU's. */
typedef struct { const uint64_t* c; const uint64_t* o; const uint8_t* b; uint64_t lo, hi; uint64_t d[4]; } tdjob;
static void* tdmain(void* a) {
  tdjob* j = (tdjob*)a;
  for (uint64_t i = j->lo; i < j->hi; i++) digest_add(j->d, j->b + j->o[i], j->o[i + 1] - j->o[i], j->c[i]);
  return NULL;
}
void moxo_table_digest(uint64_t n, const uint64_t* counts, const uint64_t* offs, const uint8_t* bytes, int nthreads,
                       uint64_t out[4]) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  tdjob jobs[64];
  pthread_t th[64];
  const uint64_t per = (n + (uint64_t)nthreads - 1) / (uint64_t)nthreads;
  for (int t = 0; t < nthreads; t++) {
    uint64_t lo = per * (uint64_t)t, hi = lo + per;
    if (lo > n) lo = n;
    if (hi > n) hi = n;
    jobs[t] = (tdjob){counts, offs, bytes, lo, hi, {0, 0, 0, 0}};
    pthread_create(&th[t], NULL, tdmain, &jobs[t]);
  }
  memset(out, 0, 4 * sizeof(uint64_t));
  for (int t = 0; t < nthreads; t++) {
    pthread_join(th[t], NULL);
    for (int k = 0; k < 4; k++) out[k] += jobs[t].d[k];
  }
}

/* Token count of s[0, n) (valid UTF-8 assumed): the cheap pass. */
typedef struct { const uint8_t* s; uint64_t n, tokens; } tcjob;
static void* tcmain(void* a) { tcjob* j = (tcjob*)a; j->tokens = for_tokens(j->s, j->n, NULL, NULL); return NULL; }
uint64_t moxo_count_tokens(const uint8_t* s, uint64_t n, int nthreads) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  uint64_t cuts[65];
  const int nt = cut_lines(s, n, nthreads, cuts);
  tcjob jobs[64];
  pthread_t th[64];
  for (int t = 0; t < nt; t++) {
    jobs[t] = (tcjob){s + cuts[t], cuts[t + 1] - cuts[t], 0};
    pthread_create(&th[t], NULL, tcmain, &jobs[t]);
  }
  uint64_t tok = 0;
  for (int t = 0; t < nt; t++) { pthread_join(th[t], NULL); tok += jobs[t].tokens; }
  return tok;
}

/* Counts of k given (lowercased) words in s[0, n): a spot check of a table. */
typedef struct { const uint8_t* s; uint64_t n; const cmap* set; uint64_t* cnt; } wcjob;
static void wc_tok(void* ctx, const uint8_t* w, uint64_t len) {
  wcjob* j = (wcjob*)ctx;
  const cmap* m = j->set;
  const uint64_t h = fnv(w, len);
  for (uint64_t k = h & (m->cap - 1);; k = (k + 1) & (m->cap - 1)) {
    const slot_t* sl = &m->slots[k];
    if (!sl->h) return;
    if (sl->h == h && sl->len == len && memcmp(m->arena + sl->off, w, len) == 0) { j->cnt[sl->count]++; return; }
  }
}
static void* wcmain(void* a) { wcjob* j = (wcjob*)a; for_tokens(j->s, j->n, wc_tok, j); return NULL; }
void moxo_count_words(const uint8_t* s, uint64_t n, int nthreads, const uint8_t* wbytes, const uint64_t* woffs, uint64_t k,
                      uint64_t* out) {
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 64) nthreads = 64;
  cmap set;  /* word -> its index (in the count field) */
  cmap_init(&set);
  for (uint64_t i = 0; i < k; i++) cmap_add(&set, wbytes + woffs[i], woffs[i + 1] - woffs[i], i);
  uint64_t cuts[65];
  const int nt = cut_lines(s, n, nthreads, cuts);
  wcjob jobs[64];
  pthread_t th[64];
  for (int t = 0; t < nt; t++) {
    jobs[t] = (wcjob){s + cuts[t], cuts[t + 1] - cuts[t], &set, (uint64_t*)calloc(k + 1, 8)};
    pthread_create(&th[t], NULL, wcmain, &jobs[t]);
  }
  memset(out, 0, k * 8);
  for (int t = 0; t < nt; t++) {
    pthread_join(th[t], NULL);
    for (uint64_t i = 0; i < k; i++) out[i] += jobs[t].cnt[i];
    free(jobs[t].cnt);
  }
  cmap_free(&set);
}
