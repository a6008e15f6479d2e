// Streaming probe for the bucket reduce's read pattern (not part of the engine).
// 1024 workgroups of 1024 threads (2 per CU, 80 KB LDS each), workgroup b reads
// 256 regions of N records (16 B) -- one per map workgroup -- 16 regions per
// wave, and xor-folds them.  Layouts of region (g, b) with capacity CAP:
//   0  g-major      (g * NB + b) * CAP            (the engine's layout)
//   1  tiled T=16   (((g / 16) * NB + b) * 16 + g % 16) * CAP
//   2  b-major      (b * G + g) * CAP
// Build: hipcc -O3 --offload-arch=gfx950 tools/probe_stream.hip -o probe_stream
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

constexpr int NB = 1024, G = 256, NWV = 16;

template <int LAYOUT, int U>
__global__ __launch_bounds__(1024, 8) void probe(const uint4* cold, uint32_t cap, uint32_t n, uint32_t* out) {
  extern __shared__ uint32_t lds[];
  const uint32_t b = blockIdx.x, lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  uint32_t acc = 0;
  for (uint32_t k = 0; k < G / NWV; k++) {
    const uint32_t g = wv + k * NWV;
    uint64_t r;
    if (LAYOUT == 0) r = (uint64_t)g * NB + b;
    else if (LAYOUT == 1) r = ((uint64_t)(g / 16) * NB + b) * 16 + g % 16;
    else r = (uint64_t)b * G + g;
    const uint4* reg = cold + r * cap;
    for (uint32_t i0 = 0; i0 < n; i0 += 64 * U) {
      uint4 v[U];
#pragma unroll
      for (int u = 0; u < U; u++) {
        const uint32_t i = i0 + u * 64 + lane;
        v[u] = reg[i < n ? i : 0];
      }
#pragma unroll
      for (int u = 0; u < U; u++) acc ^= v[u].x ^ v[u].y ^ v[u].z ^ v[u].w;
    }
  }
  if (acc == 0x12345678u) lds[threadIdx.x] = acc;  // keep the loads
  if (acc == 0x12345678u) out[0] = lds[(threadIdx.x + 1) & 1023];
}

// LDS cost probe: 2 workgroups per CU of 16 waves, each lane walks CH
// independent chains of random reads (MODE 0: ds_read_b128 of a 2432-entry
// uint4 table; MODE 1: b128 read then a u64 atomic add at the same index;
// MODE 2: as 1 but indices in 64 hot slots).  Reports LDS ops per CU-cycle.
template <int MODE, int CH>
__global__ __launch_bounds__(1024, 8) void lds_probe(uint32_t iters, uint32_t* out, unsigned long long* cyc) {
  extern __shared__ __attribute__((aligned(16))) uint8_t sm[];
  uint4* key = (uint4*)sm;
  unsigned long long* cnt = (unsigned long long*)(sm + 2432 * 16);
  for (int i = threadIdx.x; i < 2432; i += 1024) { key[i] = make_uint4(i, i * 3, i * 5, i * 7); cnt[i] = 0; }
  __syncthreads();
  uint32_t x[CH];
#pragma unroll
  for (int c = 0; c < CH; c++) x[c] = (threadIdx.x * 0x9E3779B1u) ^ (blockIdx.x * 0x85EBCA6Bu) ^ (c * 0xC2B2AE35u);
  const unsigned long long t0 = __builtin_amdgcn_s_memtime();
  for (uint32_t it = 0; it < iters; it++) {
#pragma unroll
    for (int c = 0; c < CH; c++) {
      const uint32_t idx = MODE == 2 ? (x[c] >> 8) % 64u : (x[c] >> 8) % 2432u;
      const uint4 v = key[idx];
      if (MODE >= 1) atomicAdd(&cnt[idx], 1ull);
      x[c] = (x[c] ^ v.x ^ v.w) * 0x2C1B3C6Du + 0x9E3779B9u;
    }
  }
  const unsigned long long t1 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
#pragma unroll
  for (int c = 0; c < CH; c++) acc ^= x[c];
  if (acc == 0x12345678u) out[0] = acc;
  if (threadIdx.x == 0) cyc[blockIdx.x] = t1 - t0;
}

template <int MODE, int CH>
void run_lds(uint32_t* out, unsigned long long* cyc) {
  const uint32_t iters = 512;
  lds_probe<MODE, CH><<<512, 1024, 80 * 1024>>>(iters, out, cyc);
  hipDeviceSynchronize();
  unsigned long long h[512];
  hipMemcpy(h, cyc, sizeof h, hipMemcpyDeviceToHost);
  double m = 0;
  for (int i = 0; i < 512; i++) m += h[i];
  m /= 512;
  const double ops_per_wg = (double)iters * CH * 16;  // wave-level reads per workgroup
  printf("lds mode %d chains %d: %.0f cycles per wave-read per wave (latency view), %.1f cycles per wave-read per CU (2 WGs)\n",
         MODE, CH, m / (iters * CH) * CH, m / (2 * ops_per_wg));
}

template <int L, int U>
float run(const uint4* d, uint32_t cap, uint32_t n, uint32_t* out) {
  hipEvent_t a, z;
  hipEventCreate(&a);
  hipEventCreate(&z);
  probe<L, U><<<NB, 1024, 80 * 1024>>>(d, cap, n, out);
  hipEventRecord(a);
  for (int r = 0; r < 10; r++) probe<L, U><<<NB, 1024, 80 * 1024>>>(d, cap, n, out);
  hipEventRecord(z);
  hipEventSynchronize(z);
  float ms;
  hipEventElapsedTime(&ms, a, z);
  return ms / 10;
}

int main(int argc, char** argv) {
  const uint32_t cap = argc > 1 ? atoi(argv[1]) : 512, n = argc > 2 ? atoi(argv[2]) : 154;
  uint4* d;
  uint32_t* out;
  const size_t bytes = (size_t)G * NB * cap * 16;
  if (hipMalloc(&d, bytes) != hipSuccess || hipMalloc(&out, 4) != hipSuccess) return 1;
  hipMemset(d, 1, bytes);
  const double useful = (double)G * NB * n * 16;
  auto rep = [&](const char* name, float ms) { printf("%-22s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, useful / (ms * 1e-3) / 1e12); };
  printf("cap %u records, %u per region, %.0f MB useful\n", cap, n, useful / 1e6);
  rep("g-major U1", run<0, 1>(d, cap, n, out));
  rep("g-major U2", run<0, 2>(d, cap, n, out));
  rep("g-major U4", run<0, 4>(d, cap, n, out));
  rep("tiled16 U1", run<1, 1>(d, cap, n, out));
  rep("tiled16 U2", run<1, 2>(d, cap, n, out));
  rep("tiled16 U4", run<1, 4>(d, cap, n, out));
  rep("b-major U1", run<2, 1>(d, cap, n, out));
  rep("b-major U2", run<2, 2>(d, cap, n, out));
  rep("b-major U4", run<2, 4>(d, cap, n, out));
  unsigned long long* cyc;
  hipMalloc(&cyc, 512 * 8);
  run_lds<0, 1>(out, cyc);
  run_lds<0, 4>(out, cyc);
  run_lds<1, 1>(out, cyc);
  run_lds<1, 4>(out, cyc);
  run_lds<2, 1>(out, cyc);
  run_lds<2, 4>(out, cyc);
  hipFree(d);
  return 0;
}
