/* Deterministic synthetic corpora for the word-count benchmarks.
 *
 * The reference reads a hard-coded "shakes.txt" (/root/reference/src/main.rs:10),
 * which is not shipped (.MISSING_LARGE_BLOBS:1).  The benchmark configs of
 * BASELINE.json are synthetic corpora; this file defines them byte-exactly.
 *
 * The corpus of a (kind, seed) pair is an infinite byte stream cut into 1 MiB
 * blocks.  Block b is generated from its own xoshiro256** stream seeded by
 * splitmix64(seed, b), so any byte range can be produced independently and in
 * parallel (a rank generates only its shard plus halos).  Blocks cut tokens at
 * their edges on purpose: that exercises the tile / shard word-boundary fixup.
 *
 * Kinds:
 *   ZIPF    English-like: vocabulary of 2^20 words (lengths from an English
 *           token-length distribution, mean ~4.8; letters from English letter
 *           frequencies; vocab seed 7), ranks ~ Zipf(s=1.1) (alias method);
 *           85% lower / 12% Capitalized / 3% UPPER; 8% get one trailing mark
 *           from ",.;:!?"; lines of Geometric(mean 12) tokens ending "\n"
 *           (1% "\r\n"); 1% of in-line delimiters are '\t'.
 *   HICARD  tokens of uniform length 4..16 over [a-z0-9], same line scheme.
 *   SKEW    90%: one of {the of and to a in is it that was} (9% each);
 *           10%: ZIPF vocabulary; case variants as ZIPF, no punctuation.
 *   UNICODE ZIPF words mixed with non-ASCII words (Greek with final sigma,
 *           Turkish dotted I, Kelvin sign, Cyrillic, CJK, combining marks) and
 *           multi-byte Unicode whitespace delimiters; always valid UTF-8.
 */
#include <math.h>
#include <pthread.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#define MOX_CORPUS_BLOCK (1u << 20)
#define MOX_ZIPF_V (1u << 20)

enum { MOX_CORPUS_ZIPF = 1, MOX_CORPUS_HICARD = 2, MOX_CORPUS_SKEW = 3, MOX_CORPUS_UNICODE = 4 };

typedef struct { uint64_t s[4]; } xrng;

static inline uint64_t splitmix64(uint64_t* x) {
  uint64_t z = (*x += 0x9E3779B97F4A7C15ull);
  z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
  z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
  return z ^ (z >> 31);
}
static inline uint64_t rotl64(uint64_t x, int k) { return (x << k) | (x >> (64 - k)); }
static inline uint64_t xnext(xrng* r) {
  uint64_t* s = r->s;
  uint64_t res = rotl64(s[1] * 5, 7) * 9, t = s[1] << 17;
  s[2] ^= s[0]; s[3] ^= s[1]; s[1] ^= s[2]; s[0] ^= s[3]; s[2] ^= t; s[3] = rotl64(s[3], 45);
  return res;
}
static void xseed(xrng* r, uint64_t seed, uint64_t stream) {
  uint64_t x = seed ^ (stream * 0xD1B54A32D192ED03ull);
  for (int i = 0; i < 4; i++) r->s[i] = splitmix64(&x);
}
/* uniform in [0, n) without modulo bias worth worrying about (n << 2^32) */
static inline uint32_t xbelow(xrng* r, uint32_t n) { return (uint32_t)(((xnext(r) >> 32) * (uint64_t)n) >> 32); }
static inline double xunit(xrng* r) { return (double)(xnext(r) >> 11) * (1.0 / 9007199254740992.0); }

/* ---------------- vocabulary + Zipf alias table (built once) ---------------- */
static const double LEN_W[16] = {0, .03, .17, .21, .16, .11, .08, .08, .06, .04, .03, .015, .008, .004, .002, .001};
static const char LETTERS[26] = "etaoinshrdlcumwfgypbvkjxqz";
static const double LETTER_W[26] = {12.7, 9.1, 8.2, 7.5, 7.0, 6.7, 6.3, 6.1, 6.0, 4.3, 4.0, 2.8, 2.8,
                                    2.4, 2.4, 2.2, 2.0, 2.0, 1.9, 1.5, 1.0, 0.8, 0.15, 0.15, 0.1, 0.07};

static struct {
  char* bytes;        /* concatenated words */
  uint32_t* off;      /* V+1 offsets */
  uint32_t* thresh;   /* alias probability * 2^32 */
  uint32_t* alias;
} VOC;
static pthread_once_t voc_once = PTHREAD_ONCE_INIT;

static void build_vocab(void) {
  const uint32_t V = MOX_ZIPF_V;
  xrng r; xseed(&r, 7, 0);
  double lc[16], cc[26], acc = 0, tot = 0;
  for (int i = 0; i < 16; i++) tot += LEN_W[i];
  for (int i = 0; i < 16; i++) { acc += LEN_W[i] / tot; lc[i] = acc; }
  tot = 0; acc = 0;
  for (int i = 0; i < 26; i++) tot += LETTER_W[i];
  for (int i = 0; i < 26; i++) { acc += LETTER_W[i] / tot; cc[i] = acc; }
  VOC.off = (uint32_t*)malloc((V + 1) * sizeof(uint32_t));
  VOC.bytes = (char*)malloc((size_t)V * 16);
  uint32_t o = 0;
  for (uint32_t w = 0; w < V; w++) {
    VOC.off[w] = o;
    double u = xunit(&r);
    int len = 1;
    while (len < 15 && u > lc[len]) len++;
    for (int k = 0; k < len; k++) {
      double v = xunit(&r);
      int c = 0;
      while (c < 25 && v > cc[c]) c++;
      VOC.bytes[o++] = LETTERS[c];
    }
  }
  VOC.off[V] = o;
  /* Vose alias over p_r ∝ (r+1)^-1.1 */
  double* p = (double*)malloc(V * sizeof(double));
  double H = 0;
  for (uint32_t i = 0; i < V; i++) { p[i] = exp(-1.1 * log((double)i + 1.0)); H += p[i]; }
  uint32_t *small = (uint32_t*)malloc(V * 4), *large = (uint32_t*)malloc(V * 4);
  uint32_t ns = 0, nl = 0;
  for (uint32_t i = 0; i < V; i++) { p[i] = p[i] * V / H; if (p[i] < 1.0) small[ns++] = i; else large[nl++] = i; }
  VOC.thresh = (uint32_t*)malloc(V * 4);
  VOC.alias = (uint32_t*)malloc(V * 4);
  while (ns && nl) {
    uint32_t s = small[--ns], l = large[--nl];
    VOC.thresh[s] = (uint32_t)(p[s] * 4294967295.0);
    VOC.alias[s] = l;
    p[l] = (p[l] + p[s]) - 1.0;
    if (p[l] < 1.0) small[ns++] = l; else large[nl++] = l;
  }
  while (nl) { uint32_t l = large[--nl]; VOC.thresh[l] = 0xFFFFFFFFu; VOC.alias[l] = l; }
  while (ns) { uint32_t s = small[--ns]; VOC.thresh[s] = 0xFFFFFFFFu; VOC.alias[s] = s; }
  free(p); free(small); free(large);
}

static inline uint32_t zipf_rank(xrng* r) {
  uint64_t x = xnext(r);
  uint32_t i = (uint32_t)(((x >> 32) * (uint64_t)MOX_ZIPF_V) >> 32);
  return ((uint32_t)x <= VOC.thresh[i]) ? i : VOC.alias[i];
}

/* ---------------- block writer ---------------- */
typedef struct { uint8_t* p; uint32_t n, cap; } bw;
static inline int bw_full(const bw* b) { return b->n >= b->cap; }
static inline void bw_put(bw* b, const char* s, uint32_t len) {
  uint32_t k = b->cap - b->n;
  if (len < k) k = len;
  memcpy(b->p + b->n, s, k);
  b->n += k;
}
static inline void bw_c(bw* b, char c) { if (b->n < b->cap) b->p[b->n++] = (uint8_t)c; }

static inline uint32_t geometric12(xrng* r) {
  double u = xunit(r);
  if (u <= 0) u = 1e-300;
  uint32_t k = (uint32_t)ceil(log(u) / log(1.0 - 1.0 / 12.0));
  return k < 1 ? 1 : k;
}

static void put_word_cased(bw* b, xrng* r, const char* w, uint32_t len) {
  char tmp[64];
  uint32_t u = xbelow(r, 10000);
  memcpy(tmp, w, len);
  if (u >= 9700) { for (uint32_t i = 0; i < len; i++) if (tmp[i] >= 'a' && tmp[i] <= 'z') tmp[i] -= 32; }
  else if (u >= 8500) { if (tmp[0] >= 'a' && tmp[0] <= 'z') tmp[0] -= 32; }
  bw_put(b, tmp, len);
}

static const char* HOT10[10] = {"the", "of", "and", "to", "a", "in", "is", "it", "that", "was"};
/* non-ASCII words for the UNICODE kind (UTF-8) */
static const char* UNI_WORDS[] = {
    "ΟΔΟΣ", "Σίσυφος", "ΣΑ", "σοφός", "İstanbul", "İ", "KELVIN", "\xE2\x84\xAA" "elvin", "Straße", "STRASSE",
    "МОСКВА", "москва", "Привет,", "日本語", "東京", "café", "CAFÉ", "naïve", "Ǆemal", "ǅ", "ǆ", "ΆΈΉ", "ꙊꙋⰀ",
    "e\xCC\x81", "E\xCC\x81", "x\xE2\x80\x8By", "\xEF\xBB\xBF" "The", "Σ.", "ΑΣ'Σ", "a\xC2\xADΣ", "𝔘𝔫𝔦", "😀smile"};
static const char* UNI_WS[] = {"\xC2\xA0", "\xE3\x80\x80", "\xE2\x80\x83", "\xC2\x85", "\xE2\x80\xA8", "\xE1\x9A\x80",
                               "\xE2\x80\xAF", "\xE2\x81\x9F", "\x0B", "\x0C", "\x1C"};

static void gen_block(int kind, uint64_t seed, uint64_t blk, uint8_t* out) {
  xrng r; xseed(&r, seed, blk + 1);
  bw b = {out, 0, MOX_CORPUS_BLOCK};
  uint32_t line_left = geometric12(&r);
  char tmp[32];
  static const char ALNUM[36] = "abcdefghijklmnopqrstuvwxyz0123456789";
  static const char PUNCT[6] = {',', '.', ';', ':', '!', '?'};
  const uint32_t n_uni = (uint32_t)(sizeof(UNI_WORDS) / sizeof(UNI_WORDS[0]));
  const uint32_t n_uws = (uint32_t)(sizeof(UNI_WS) / sizeof(UNI_WS[0]));
  while (!bw_full(&b)) {
    if (kind == MOX_CORPUS_HICARD) {
      uint32_t len = 4 + xbelow(&r, 13);
      for (uint32_t i = 0; i < len; i++) tmp[i] = ALNUM[xbelow(&r, 36)];
      bw_put(&b, tmp, len);
    } else if (kind == MOX_CORPUS_SKEW) {
      if (xbelow(&r, 100) < 90) {
        const char* w = HOT10[xbelow(&r, 10)];
        put_word_cased(&b, &r, w, (uint32_t)strlen(w));
      } else {
        uint32_t k = zipf_rank(&r);
        put_word_cased(&b, &r, VOC.bytes + VOC.off[k], VOC.off[k + 1] - VOC.off[k]);
      }
    } else {
      if (kind == MOX_CORPUS_UNICODE && xbelow(&r, 100) < 25) {
        const char* w = UNI_WORDS[xbelow(&r, n_uni)];
        bw_put(&b, w, (uint32_t)strlen(w));
      } else {
        uint32_t k = zipf_rank(&r);
        put_word_cased(&b, &r, VOC.bytes + VOC.off[k], VOC.off[k + 1] - VOC.off[k]);
      }
      if (xbelow(&r, 100) < 8) bw_c(&b, PUNCT[xbelow(&r, 6)]);
    }
    if (--line_left == 0) {
      if (xbelow(&r, 100) == 0) bw_c(&b, '\r');
      bw_c(&b, '\n');
      line_left = geometric12(&r);
    } else if (kind == MOX_CORPUS_UNICODE && xbelow(&r, 100) < 10) {
      const char* s = UNI_WS[xbelow(&r, n_uws)];
      bw_put(&b, s, (uint32_t)strlen(s));
    } else {
      bw_c(&b, xbelow(&r, 100) == 0 ? '\t' : ' ');
    }
  }
  /* UNICODE kind: never leave a truncated multi-byte sequence at the block end;
   * the cut lands inside a char only if the last char started in this block. */
  if (kind == MOX_CORPUS_UNICODE) {
    uint32_t n = MOX_CORPUS_BLOCK, i = n;
    while (i > 0 && n - i < 4 && (out[i - 1] & 0xC0) == 0x80) i--;
    if (i > 0 && out[i - 1] >= 0xC0) {
      uint8_t c = out[i - 1];
      uint32_t need = c >= 0xF0 ? 4 : c >= 0xE0 ? 3 : 2;
      if (n - (i - 1) < need)
        for (uint32_t k = i - 1; k < n; k++) out[k] = ' ';
    }
  }
}

typedef struct {
  int kind;
  uint64_t seed, offset, nbytes;
  uint8_t* out;
  uint64_t b0, b1;
  int tid, nthreads;
} job_t;

static void* worker(void* arg) {
  job_t* j = (job_t*)arg;
  uint8_t* buf = (uint8_t*)malloc(MOX_CORPUS_BLOCK);
  for (uint64_t blk = j->b0 + (uint64_t)j->tid; blk < j->b1; blk += (uint64_t)j->nthreads) {
    uint64_t bs = blk * MOX_CORPUS_BLOCK, be = bs + MOX_CORPUS_BLOCK;
    uint64_t lo = bs > j->offset ? bs : j->offset;
    uint64_t hi = be < j->offset + j->nbytes ? be : j->offset + j->nbytes;
    if (lo >= hi) continue;
    if (lo == bs && hi == be) {
      gen_block(j->kind, j->seed, blk, j->out + (bs - j->offset));
    } else {
      gen_block(j->kind, j->seed, blk, buf);
      memcpy(j->out + (lo - j->offset), buf + (lo - bs), hi - lo);
    }
  }
  free(buf);
  return NULL;
}

/* Fill out[0..nbytes) with bytes [offset, offset+nbytes) of corpus (kind, seed).
 * Returns 0, or -1 for an unknown kind. */
int mox_corpus_fill(int kind, uint64_t seed, uint64_t offset, uint64_t nbytes, uint8_t* out, int nthreads) {
  if (kind < MOX_CORPUS_ZIPF || kind > MOX_CORPUS_UNICODE) return -1;
  if (nbytes == 0) return 0;
  pthread_once(&voc_once, build_vocab);
  if (nthreads < 1) nthreads = 1;
  if (nthreads > 256) nthreads = 256;
  uint64_t b0 = offset / MOX_CORPUS_BLOCK, b1 = (offset + nbytes + MOX_CORPUS_BLOCK - 1) / MOX_CORPUS_BLOCK;
  if ((uint64_t)nthreads > b1 - b0) nthreads = (int)(b1 - b0);
  pthread_t th[256];
  job_t jobs[256];
  for (int t = 0; t < nthreads; t++) {
    jobs[t] = (job_t){kind, seed, offset, nbytes, out, b0, b1, t, nthreads};
    if (nthreads == 1) worker(&jobs[t]);
    else pthread_create(&th[t], NULL, worker, &jobs[t]);
  }
  if (nthreads > 1)
    for (int t = 0; t < nthreads; t++) pthread_join(th[t], NULL);
  return 0;
}

/* The vocabulary entry of Zipf rank r (for tests / docs). */
int mox_corpus_vocab_word(uint32_t rank, char* out, int cap) {
  pthread_once(&voc_once, build_vocab);
  if (rank >= MOX_ZIPF_V) return -1;
  int len = (int)(VOC.off[rank + 1] - VOC.off[rank]);
  if (len > cap) return -1;
  memcpy(out, VOC.bytes + VOC.off[rank], (size_t)len);
  return len;
}
