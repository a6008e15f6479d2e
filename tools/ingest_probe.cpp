// Ingest probe: what bounds mox_count_file on the GPU box?
//   A  pread of a page-cached file into pinned buffers, T threads (no GPU copy)
//   B  H2D copies from pinned host memory, S streams (no file reads)
//   C  both: T readers, each pread -> its own pinned double buffer -> own stream,
//      waiting only for the copy of the buffer it refills (per-buffer events)
//   D  one hipMemcpy from a pageable (malloc) 1 GiB buffer
//   E  like C, but each chunk is mmap'ed (MAP_POPULATE) and copied into the
//      pinned buffer with non-temporal 16-byte stores (the CPU leaves no dirty
//      lines for the DMA engine to snoop)
//   F  like C, but pread into the pinned buffer is followed by a cache flush-free
//      path: each chunk's pages registered (hipHostRegister of the mmap'ed chunk)
//      and copied straight from the page cache, no CPU copy
//   G  one hipMemcpy from a MAP_POPULATE mmap of the whole file (runtime staging)
// Build: hipcc -O2 -std=c++17 tools/ingest_probe.cpp -o build/ingest_probe -lpthread
// Run:   build/ingest_probe FILE [MiB]   (FILE is written first if absent)
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <emmintrin.h>
#include <sys/mman.h>
#include <unistd.h>
#include <atomic>
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
  // E: mmap + non-temporal copy into pinned + H2D (shared stream)
  auto nt_copy = [](uint8_t* dst, const uint8_t* src, size_t n) {
    size_t i = 0;
    for (; i + 64 <= n; i += 64) {
      __m128i a = _mm_loadu_si128((const __m128i*)(src + i)), b = _mm_loadu_si128((const __m128i*)(src + i + 16));
      __m128i c = _mm_loadu_si128((const __m128i*)(src + i + 32)), d = _mm_loadu_si128((const __m128i*)(src + i + 48));
      _mm_stream_si128((__m128i*)(dst + i), a); _mm_stream_si128((__m128i*)(dst + i + 16), b);
      _mm_stream_si128((__m128i*)(dst + i + 32), c); _mm_stream_si128((__m128i*)(dst + i + 48), d);
    }
    for (; i < n; i++) dst[i] = src[i];
    _mm_sfence();
  };
  for (int shared : {1, 0}) for (int T : {8, 16}) {
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
        hipStream_t cs = st[shared ? 0 : t];
        for (size_t c = t; c < nch; c += T, k ^= 1) {
          if (used[k]) (void)hipEventSynchronize(ev[k]);
          const size_t n = std::min(CH, len - c * CH);
          void* m = mmap(nullptr, n, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, (off_t)(c * CH));
          if (m == MAP_FAILED) exit(4);
          nt_copy(pin[2 * t + k], (const uint8_t*)m, n);
          munmap(m, n);
          (void)hipMemcpyAsync(d + c * CH, pin[2 * t + k], n, hipMemcpyHostToDevice, cs);
          (void)hipEventRecord(ev[k], cs);
          used[k] = true;
        }
        (void)hipStreamSynchronize(cs);
        for (auto& e : ev) (void)hipEventDestroy(e);
      });
      for (auto& x : th) x.join();
      CK(hipDeviceSynchronize());
      best = std::min(best, now_s() - t0);
    }
    printf("E mmap+nt+H2D %s T=%2d  %.1f GB/s\n", shared ? "1 stream " : "T streams", T, len / best / 1e9);
  }
  // E2: pread + H2D, shared stream (the engine's scheme), for reference
  for (int T : {8, 16}) {
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
          (void)hipMemcpyAsync(d + c * CH, pin[2 * t + k], n, hipMemcpyHostToDevice, st[0]);
          (void)hipEventRecord(ev[k], st[0]);
          used[k] = true;
        }
        for (auto& e : ev) (void)hipEventDestroy(e);
      });
      for (auto& x : th) x.join();
      CK(hipDeviceSynchronize());
      best = std::min(best, now_s() - t0);
    }
    printf("E2 pread+H2D 1 stream T=%2d  %.1f GB/s\n", T, len / best / 1e9);
  }
  // F: mmap + hipHostRegister per chunk, H2D straight from the page cache
  for (int T : {4, 8}) {
    double best = 1e9;
    bool ok = true;
    for (int rep = 0; rep < 3 && ok; rep++) {
      CK(hipDeviceSynchronize());
      const double t0 = now_s();
      std::vector<std::thread> th;
      std::atomic<bool> bad{false};
      for (int t = 0; t < T; t++) th.emplace_back([&, t] {
        (void)hipSetDevice(0);
        for (size_t c = t; c < nch; c += T) {
          const size_t n = std::min(CH, len - c * CH);
          void* m = mmap(nullptr, n, PROT_READ, MAP_SHARED | MAP_POPULATE, fd, (off_t)(c * CH));
          if (m == MAP_FAILED) { bad = true; return; }
          if (hipHostRegister(m, n, hipHostRegisterReadOnly) != hipSuccess) { bad = true; munmap(m, n); return; }
          (void)hipMemcpyAsync(d + c * CH, m, n, hipMemcpyHostToDevice, st[t]);
          (void)hipStreamSynchronize(st[t]);
          (void)hipHostUnregister(m);
          munmap(m, n);
        }
      });
      for (auto& x : th) x.join();
      if (bad) { ok = false; break; }
      best = std::min(best, now_s() - t0);
    }
    if (ok) printf("F mmap+register T=%2d  %.1f GB/s\n", T, len / best / 1e9);
    else printf("F mmap+register T=%2d  failed (hipHostRegister refused the file mapping)\n", T);
  }
  // G: one hipMemcpy from a populated mmap of the whole file
  {
    double best = 1e9;
    for (int rep = 0; rep < 3; rep++) {
      const double t0 = now_s();
      void* m = mmap(nullptr, len, PROT_READ, MAP_PRIVATE | MAP_POPULATE, fd, 0);
      if (m == MAP_FAILED) exit(5);
      CK(hipMemcpy(d, m, len, hipMemcpyHostToDevice));
      munmap(m, len);
      best = std::min(best, now_s() - t0);
    }
    printf("G mmap whole + hipMemcpy  %.1f GB/s\n", len / best / 1e9);
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
