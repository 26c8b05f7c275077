// H2D bandwidth on one MI355X for the engine's sources: hipHostMalloc'd pinned memory vs a
// shared-memory mapping page-locked with hipHostRegister (the rings), one copy vs the same
// bytes split over k streams (several SDMA engines). Prints GB/s per case.
#include <hip/hip_runtime.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <unistd.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#define CK(x)                                                                       \
  do {                                                                              \
    hipError_t e = (x);                                                             \
    if (e != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                   \
      return 1;                                                                     \
    }                                                                               \
  } while (0)

static double run(const uint8_t* src, uint8_t* dst, size_t n, int k, std::vector<hipStream_t>& st, int reps) {
  const size_t q = (n / k) & ~size_t(4095);
  auto once = [&] {
    for (int j = 0; j < k; ++j) {
      const size_t lo = j * q, hi = j == k - 1 ? n : (j + 1) * q;
      (void)hipMemcpyAsync(dst + lo, src + lo, hi - lo, hipMemcpyHostToDevice, st[j]);
    }
    for (int j = 0; j < k; ++j) (void)hipStreamSynchronize(st[j]);
  };
  for (int i = 0; i < 3; ++i) once();
  const auto t0 = std::chrono::steady_clock::now();
  for (int i = 0; i < reps; ++i) once();
  const double s = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  return reps * (double)n / s / 1e9;
}

int main() {
  const size_t n = 32u << 20;
  CK(hipSetDevice(0));
  std::vector<hipStream_t> st(8);
  for (auto& s : st) CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  uint8_t* d = nullptr;
  CK(hipMalloc(&d, n));
  void* pinned = nullptr;
  CK(hipHostMalloc(&pinned, n, hipHostMallocDefault));
  std::memset(pinned, 1, n);
  const char* name = "/mislo-h2d-bw";
  shm_unlink(name);
  int fd = shm_open(name, O_CREAT | O_RDWR, 0600);
  if (fd < 0 || ftruncate(fd, n) != 0) return 1;
  void* shm = mmap(nullptr, n, PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  if (shm == MAP_FAILED) return 1;
  std::memset(shm, 2, n);
  CK(hipHostRegister(shm, n, hipHostRegisterDefault));
  for (int k : {1, 2, 3, 4}) {
    std::printf("32 MiB  %d stream(s): hipHostMalloc %6.1f GB/s   registered shm %6.1f GB/s\n", k,
                run((const uint8_t*)pinned, d, n, k, st, 30), run((const uint8_t*)shm, d, n, k, st, 30));
    std::fflush(stdout);
  }
  CK(hipHostUnregister(shm));
  munmap(shm, n);
  close(fd);
  shm_unlink(name);
  (void)hipHostFree(pinned);
  (void)hipFree(d);
  return 0;
}
