// Ingest probe: what bounds mox_count_file on the GPU box?
//   A  pread of a page-cached file into pinned buffers, T threads (no GPU copy)
//   B  H2D copies from pinned host memory, S streams (no file reads)
//   C  both: T readers, each pread -> its own pinned double buffer -> own stream,
//      waiting only for the copy of the buffer it refills (per-buffer events)
//   D  one hipMemcpy from a pageable (malloc) 1 GiB buffer
// Build: hipcc -O2 -std=c++17 tools/ingest_probe.cpp -o build/ingest_probe -lpthread
// Run:   build/ingest_probe FILE [MiB]   (FILE is written first if absent)
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <unistd.h>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <thread>
#include <vector>

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); exit(1); } } while (0)

static double now_s() { return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count(); }

int main(int argc, char** argv) {
  if (argc < 2) { fprintf(stderr, "usage: %s FILE [MiB]\n", argv[0]); return 2; }
  const size_t len = (size_t)(argc > 2 ? atol(argv[2]) : 1024) << 20;
  int fd = open(argv[1], O_RDONLY);
  if (fd < 0) {  // write a text-like file (page cache keeps it)
    int wf = open(argv[1], O_WRONLY | O_CREAT | O_TRUNC, 0644);
    std::vector<char> blk(1 << 20);
    for (size_t i = 0; i < blk.size(); i++) blk[i] = (i % 7 == 6) ? ' ' : (char)('a' + (i * 131 % 26));
    for (size_t o = 0; o < len; o += blk.size()) if (write(wf, blk.data(), blk.size()) < 0) return 1;
    close(wf);
    fd = open(argv[1], O_RDONLY);
  }
  uint8_t* d = nullptr;
  CK(hipMalloc((void**)&d, len));
  const size_t CH = 32 << 20;
  const size_t nch = (len + CH - 1) / CH;
  std::vector<uint8_t*> pin(2 * 32);
  for (auto& p : pin) CK(hipHostMalloc((void**)&p, CH, hipHostMallocDefault));
  std::vector<hipStream_t> st(32);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  auto rd = [&](uint8_t* dst, size_t off, size_t n) {
    size_t got = 0;
    while (got < n) { ssize_t r = pread(fd, dst + got, n - got, (off_t)(off + got)); if (r <= 0) exit(3); got += (size_t)r; }
  };
  // A: pread only
  for (int T : {4, 8, 16, 24}) {
    double best = 1e9;
    for (int rep = 0; rep < 3; rep++) {
      const double t0 = now_s();
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++) th.emplace_back([&, t] {
        int k = 0;
        for (size_t c = t; c < nch; c += T, k ^= 1) rd(pin[2 * t + k], c * CH, std::min(CH, len - c * CH));
      });
      for (auto& x : th) x.join();
      best = std::min(best, now_s() - t0);
    }
    printf("A pread only      T=%2d  %.1f GB/s\n", T, len / best / 1e9);
  }
  // B: H2D only from pinned buffers
  for (int S : {1, 2, 4, 8}) {
    double best = 1e9;
    for (int rep = 0; rep < 3; rep++) {
      CK(hipDeviceSynchronize());
      const double t0 = now_s();
      for (size_t c = 0; c < nch; c++) CK(hipMemcpyAsync(d + c * CH, pin[c % 64], std::min(CH, len - c * CH), hipMemcpyHostToDevice, st[c % S]));
      CK(hipDeviceSynchronize());
      best = std::min(best, now_s() - t0);
    }
    printf("B H2D pinned      S=%2d  %.1f GB/s\n", S, len / best / 1e9);
  }
  // C: pread -> pinned -> H2D, per-buffer events
  for (int T : {8, 12, 16}) {
    double best = 1e9;
    for (int rep = 0; rep < 3; rep++) {
      CK(hipDeviceSynchronize());
      const double t0 = now_s();
      std::vector<std::thread> th;
      for (int t = 0; t < T; t++) th.emplace_back([&, t] {
        (void)hipSetDevice(0);
        hipEvent_t ev[2];
        for (auto& e : ev) (void)hipEventCreateWithFlags(&e, hipEventDisableTiming);
        bool used[2] = {false, false};
        int k = 0;
        for (size_t c = t; c < nch; c += T, k ^= 1) {
          if (used[k]) (void)hipEventSynchronize(ev[k]);
          const size_t n = std::min(CH, len - c * CH);
          rd(pin[2 * t + k], c * CH, n);
          (void)hipMemcpyAsync(d + c * CH, pin[2 * t + k], n, hipMemcpyHostToDevice, st[t]);
          (void)hipEventRecord(ev[k], st[t]);
          used[k] = true;
        }
        (void)hipStreamSynchronize(st[t]);
        for (auto& e : ev) (void)hipEventDestroy(e);
      });
      for (auto& x : th) x.join();
      best = std::min(best, now_s() - t0);
    }
    printf("C pread+H2D       T=%2d  %.1f GB/s\n", T, len / best / 1e9);
  }
  // D: pageable hipMemcpy
  {
    std::vector<uint8_t> h(len);
    rd(h.data(), 0, len);
    double best = 1e9;
    for (int rep = 0; rep < 3; rep++) {
      const double t0 = now_s();
      CK(hipMemcpy(d, h.data(), len, hipMemcpyHostToDevice));
      best = std::min(best, now_s() - t0);
    }
    printf("D H2D pageable          %.1f GB/s\n", len / best / 1e9);
  }
  return 0;
}
