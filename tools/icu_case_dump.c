/* ICU 70 case-data probe for tools/icu_pin.py (test-fixture generator; not part
 * of the product path).  Build: gcc -O2 tools/icu_case_dump.c -licuuc -o <out>
 *
 *   icu_case_dump --table   one line per code point whose lowercase differs from
 *                           itself or that is Cased / Case_Ignorable / White_Space:
 *                           "cp age lower flags" -- cp hex, age "M.m" (u_charAge),
 *                           lower = u_strToLower(root locale "") of the code point
 *                           alone as '.'-joined hex, flags C (Cased), I
 *                           (Case_Ignorable), W (White_Space) or '-'.
 *   icu_case_dump --strings reads hex-encoded UTF-8 strings, one per line, and
 *                           prints u_strToLower(root) of each, hex UTF-8 -- this
 *                           exercises the contextual Final_Sigma rule.
 *   icu_case_dump --age     reads hex code points, one per line, prints u_charAge "M.m".
 */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unicode/uchar.h>
#include <unicode/ustring.h>
#include <unicode/uversion.h>

static int lower_utf16(const UChar* src, int32_t n, UChar* dst, int32_t cap) {
  UErrorCode st = U_ZERO_ERROR;
  int32_t m = u_strToLower(dst, cap, src, n, "", &st);
  if (U_FAILURE(st)) {
    fprintf(stderr, "u_strToLower: %s\n", u_errorName(st));
    exit(1);
  }
  return m;
}

static int table(void) {
  UVersionInfo uv;
  u_getUnicodeVersion(uv);
  printf("# unicode %d.%d.%d icu %s\n", uv[0], uv[1], uv[2], U_ICU_VERSION);
  for (UChar32 cp = 0; cp <= 0x10FFFF; cp++) {
    if (cp >= 0xD800 && cp <= 0xDFFF) continue;
    UChar src[2], dst[16];
    int32_t n = 0;
    U16_APPEND_UNSAFE(src, n, cp);
    int32_t m = lower_utf16(src, n, dst, 16);
    int same = (m == n) && memcmp(src, dst, n * sizeof(UChar)) == 0;
    int c = u_hasBinaryProperty(cp, UCHAR_CASED), ci = u_hasBinaryProperty(cp, UCHAR_CASE_IGNORABLE);
    int ws = u_hasBinaryProperty(cp, UCHAR_WHITE_SPACE);
    if (same && !c && !ci && !ws) continue;
    UVersionInfo age;
    u_charAge(cp, age);
    printf("%x %d.%d ", cp, age[0], age[1]);
    for (int32_t i = 0; i < m;) {
      UChar32 o;
      U16_NEXT(dst, i, m, o);
      printf(i == m ? "%x" : "%x.", o);
    }
    printf(" %s%s%s%s\n", c ? "C" : "", ci ? "I" : "", ws ? "W" : "", (c || ci || ws) ? "" : "-");
  }
  return 0;
}

static int strings(void) {
  static char line[1 << 16];
  static unsigned char u8[1 << 15], o8[1 << 17];
  static UChar u16[1 << 15], l16[1 << 17];
  while (fgets(line, sizeof line, stdin)) {
    size_t hl = strcspn(line, "\r\n"), n = hl / 2;
    for (size_t i = 0; i < n; i++) {
      unsigned v;
      sscanf(line + 2 * i, "%2x", &v);
      u8[i] = (unsigned char)v;
    }
    UErrorCode st = U_ZERO_ERROR;
    int32_t n16 = 0, m8 = 0;
    u_strFromUTF8(u16, 1 << 15, &n16, (const char*)u8, (int32_t)n, &st);
    if (U_FAILURE(st)) { fprintf(stderr, "u_strFromUTF8: %s\n", u_errorName(st)); return 1; }
    int32_t m16 = lower_utf16(u16, n16, l16, 1 << 17);
    u_strToUTF8((char*)o8, 1 << 17, &m8, l16, m16, &st);
    if (U_FAILURE(st)) { fprintf(stderr, "u_strToUTF8: %s\n", u_errorName(st)); return 1; }
    for (int32_t i = 0; i < m8; i++) printf("%02x", o8[i]);
    printf("\n");
  }
  return 0;
}

static int ages(void) {
  unsigned cp;
  while (scanf("%x", &cp) == 1) {
    UVersionInfo age;
    u_charAge((UChar32)cp, age);
    printf("%d.%d\n", age[0], age[1]);
  }
  return 0;
}

int main(int argc, char** argv) {
  if (argc == 2 && !strcmp(argv[1], "--table")) return table();
  if (argc == 2 && !strcmp(argv[1], "--strings")) return strings();
  if (argc == 2 && !strcmp(argv[1], "--age")) return ages();
  fprintf(stderr, "usage: %s --table | --strings | --age\n", argv[0]);
  return 2;
}
