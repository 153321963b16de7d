// modinv_check.cpp -- host check of p256_modinv.h (tools only): prints "x inv" hex pairs for
// edge cases + xorshift-random inputs; tools/modinv_check.py verifies x*inv == 1 mod n.
#define FGV_HD inline
#include <cstdio>
#include <cstdlib>

#include "../fabric_amd/csrc/p256_modinv.h"

static uint64_t st = 0x9E3779B97F4A7C15ull;
static uint32_t rnd() {
  st ^= st << 13;
  st ^= st >> 7;
  st ^= st << 17;
  return (uint32_t)(st >> 16);
}
static void emit(const uint32_t x[8]) {
  uint32_t r[8];
  fgv_modinv::modinv_n(r, x);
  for (int i = 7; i >= 0; i--) printf("%08x", x[i]);
  printf(" ");
  for (int i = 7; i >= 0; i--) printf("%08x", r[i]);
  printf("\n");
}
int main(int argc, char **argv) {
  const int count = argc > 1 ? atoi(argv[1]) : 100000;
  const uint32_t N[8] = {0xFC632551u, 0xF3B9CAC2u, 0xA7179E84u, 0xBCE6FAADu, 0xFFFFFFFFu, 0xFFFFFFFFu, 0u, 0xFFFFFFFFu};
  uint32_t x[8];
  // edge cases: 1, 2, n-1, n-2, (n-1)/2, 2^k, all-ones below n
  for (int k = 0; k < 256; k++) {
    for (int i = 0; i < 8; i++) x[i] = 0;
    x[k >> 5] = 1u << (k & 31);
    bool lt = false;
    for (int i = 7; i >= 0; i--)
      if (x[i] != N[i]) { lt = x[i] < N[i]; break; }
    if (lt) emit(x);
  }
  for (int d = 1; d <= 3; d++) {
    uint32_t b = 0;
    for (int i = 0; i < 8; i++) {
      uint64_t t = (uint64_t)N[i] - (i == 0 ? d : 0) - b;
      x[i] = (uint32_t)t;
      b = (t >> 63) & 1;
    }
    emit(x);
  }
  for (int c = 0; c < count; c++) {
    for (int i = 0; i < 8; i++) x[i] = rnd();
    const int mode = c % 4;
    if (mode == 1) x[7] = 0;                    // small-ish
    if (mode == 2) for (int i = 4; i < 8; i++) x[i] = 0xFFFFFFFFu;  // near 2^256 (reduced below)
    if (mode == 3) for (int i = 1; i < 8; i++) x[i] = 0;            // tiny
    bool ge = true;
    for (int i = 7; i >= 0; i--)
      if (x[i] != N[i]) { ge = x[i] > N[i]; break; }
    if (ge) x[7] = 0x7FFFFFFFu;
    bool zero = true;
    for (int i = 0; i < 8; i++) zero &= x[i] == 0;
    if (zero) x[0] = 1;
    emit(x);
  }
  return 0;
}
