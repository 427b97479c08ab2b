// Host build of ar_orbslam2_amd/csrc/orbx_math.h checked against the host libm sincosf over
// every float in [lo, hi] and against the oracle's fastAtan2 on integer moment pairs.
// Test infrastructure (tests/test_math_port.py builds and runs it).
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <pthread.h>
#include <stdint.h>
#include "../../ar_orbslam2_amd/csrc/orbx_math.h"

static uint32_t g_lo, g_hi;
static uint64_t g_bad[64];
static int g_nt;
static void* work(void* a) {
  long t = (long)a;
  for (uint64_t u = (uint64_t)g_lo + t; u <= g_hi; u += g_nt) {
    uint32_t v = (uint32_t)u;
    float f;
    memcpy(&f, &v, 4);
    float s, c, s2, c2;
    sincosf(f, &s, &c);
    orbx::orbx_sincosf(f, &s2, &c2);
    if (memcmp(&s, &s2, 4) || memcmp(&c, &c2, 4)) g_bad[t]++;
  }
  return 0;
}
int main(int argc, char** argv) {
  g_lo = (uint32_t)strtoul(argv[1], 0, 0);
  g_hi = (uint32_t)strtoul(argv[2], 0, 0);
  g_nt = argc > 3 ? atoi(argv[3]) : 8;
  pthread_t th[64];
  for (long t = 0; t < g_nt; t++) pthread_create(&th[t], 0, work, (void*)t);
  uint64_t bad = 0;
  for (int t = 0; t < g_nt; t++) pthread_join(th[t], 0), bad += g_bad[t];
  printf("sincosf_mismatches %llu\n", (unsigned long long)bad);
  return bad != 0;
}
