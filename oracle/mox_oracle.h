/* ORACLE -- test infrastructure only (see mox_oracle.c header).  PARITY UNPINNED. */
#pragma once
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MOXO_EUTF8 (-2)

typedef struct {
  uint64_t n;          /* unique words */
  uint64_t tokens;     /* total tokens */
  uint64_t* counts;    /* n */
  uint64_t* offs;      /* n+1, into bytes */
  uint8_t* bytes;      /* words, sorted bytewise ascending */
  uint64_t bytes_len;
  int64_t invalid_at;  /* first invalid UTF-8 byte, or -1 */
} moxo_table;

int moxo_count(const uint8_t* text, uint64_t len, int nthreads, moxo_table* out);
int moxo_count_range(const uint8_t* text, uint64_t len, uint64_t own_begin, uint64_t own_end, moxo_table* out);
void moxo_free(moxo_table* t);
int64_t moxo_utf8_invalid_at(const uint8_t* s, uint64_t n);
int moxo_is_whitespace(uint32_t c);
uint64_t moxo_lowercase(const uint8_t* s, uint64_t n, uint8_t* out);
/* property checks for big corpora (no sorted table) */
int moxo_count_digest(const uint8_t* s, uint64_t n, int nthreads, uint64_t out[4], uint64_t* tokens);
void moxo_table_digest(uint64_t n, const uint64_t* counts, const uint64_t* offs, const uint8_t* bytes, int nthreads,
                       uint64_t out[4]);
uint64_t moxo_count_tokens(const uint8_t* s, uint64_t n, int nthreads);
void moxo_count_words(const uint8_t* s, uint64_t n, int nthreads, const uint8_t* wbytes, const uint64_t* woffs, uint64_t k,
                      uint64_t* out);

#ifdef __cplusplus
}
#endif
