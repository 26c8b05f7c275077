// Host-memory floor of the HIP runtime on MI355X: RSS and the large resident anonymous
// mappings after each step of bringing up a device the way the agent's engine does (no torch,
// no extension), so the agent's RSS can be split into what HIP itself maps and what the
// engine adds. Build: hipcc --offload-arch=gfx950 -O2 tools/native/hip_rss_floor.hip -o build/hip_rss_floor
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

__constant__ float c_tab[1024];

__global__ void k_touch(float* p, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) p[i] = c_tab[i & 1023] + 1.f;
}

static double rss_mb() {
  FILE* f = fopen("/proc/self/statm", "r");
  long a = 0, b = 0;
  if (f) {
    if (fscanf(f, "%ld %ld", &a, &b) != 2) b = 0;
    fclose(f);
  }
  return b * 4096.0 / 1048576.0;
}

// resident mappings >= 8 MB: name (or [anon]), size, rss
static void big_maps() {
  FILE* f = fopen("/proc/self/smaps", "r");
  if (!f) return;
  char ln[4096];
  std::string name;
  double size = 0;
  while (fgets(ln, sizeof ln, f)) {
    unsigned long a, b;
    char perm[8];
    int off = 0;
    if (sscanf(ln, "%lx-%lx %7s %*s %*s %*s %n", &a, &b, perm, &off) >= 3 && strchr(ln, '-') < strchr(ln, ' ')) {
      name = off > 0 && ln[off] && ln[off] != '\n' ? std::string(ln + off) : std::string("[anon]\n");
      name.pop_back();
      size = (b - a) / 1048576.0;
      name += std::string(" ") + perm;
    } else if (!strncmp(ln, "Rss:", 4)) {
      const double r = atol(ln + 4) / 1024.0;
      if (r >= 8.0) printf("      %8.1f MB rss of %8.1f MB  %s\n", r, size, name.c_str());
    }
  }
  fclose(f);
}

static void step(const char* what, hipError_t e = hipSuccess) {
  if (e != hipSuccess) {
    printf("%-36s FAILED %s\n", what, hipGetErrorString(e));
    exit(1);
  }
  printf("%-36s rss %8.1f MB\n", what, rss_mb());
  big_maps();
  fflush(stdout);
}

int main() {
  step("start");
  step("hipInit", hipInit(0));
  int n = 0;
  step("hipGetDeviceCount", hipGetDeviceCount(&n));
  step("hipSetDevice", hipSetDevice(0));
  step("hipFree(0) (context)", hipFree(nullptr));
  hipStream_t s;
  step("hipStreamCreateWithFlags", hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
  float* d = nullptr;
  step("hipMalloc 64 MB", hipMalloc(&d, 64 << 20));
  std::vector<float> h(1024, 1.f);
  step("hipMemcpyToSymbol (constant table)", hipMemcpyToSymbol(HIP_SYMBOL(c_tab), h.data(), sizeof(float) * 1024));
  k_touch<<<1024, 256, 0, s>>>(d, 1 << 18);
  step("first kernel launch", hipGetLastError());
  step("hipStreamSynchronize", hipStreamSynchronize(s));
  step("hipMemcpyAsync D2H 4 KB", hipMemcpyAsync(h.data(), d, 4096, hipMemcpyDeviceToHost, s));
  step("hipStreamSynchronize", hipStreamSynchronize(s));
  void* pin = nullptr;
  step("hipHostMalloc 16 MB", hipHostMalloc(&pin, 16 << 20, hipHostMallocDefault));
  hipGraph_t g;
  hipGraphExec_t ge;
  step("begin capture", hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
  k_touch<<<1024, 256, 0, s>>>(d, 1 << 18);
  step("end capture", hipStreamEndCapture(s, &g));
  step("hipGraphInstantiate", hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
  step("hipGraphLaunch", hipGraphLaunch(ge, s));
  step("hipStreamSynchronize", hipStreamSynchronize(s));
  // the engine's per-window calls, one at a time: which of them maps a queue save area beyond
  // the stream's (round 5: the agent holds three 173.4 MB areas at GPU_MAX_HW_QUEUES=1)
  step("hipMemcpyAsync H2D 16 MB pinned", hipMemcpyAsync(d, pin, 16 << 20, hipMemcpyHostToDevice, s));
  step("hipStreamSynchronize", hipStreamSynchronize(s));
  std::vector<char> big(32 << 20, 1);
  step("hipHostRegister 32 MB", hipHostRegister(big.data(), big.size(), hipHostRegisterDefault));
  step("hipMemcpyAsync H2D 32 MB registered", hipMemcpyAsync(d, big.data(), 32 << 20, hipMemcpyHostToDevice, s));
  step("hipStreamSynchronize", hipStreamSynchronize(s));
  hipEvent_t ev;
  step("hipEventCreateWithFlags", hipEventCreateWithFlags(&ev, hipEventDisableTiming));
  step("hipEventRecord", hipEventRecord(ev, s));
  step("hipEventSynchronize", hipEventSynchronize(ev));
  hipEvent_t evt;
  step("hipEventCreate (timing)", hipEventCreate(&evt));
  step("hipEventRecord (timing)", hipEventRecord(evt, s));
  step("hipEventSynchronize (timing)", hipEventSynchronize(evt));
  step("hipMemcpy D2H 8 B (null stream)", hipMemcpy(h.data(), d, 8, hipMemcpyDeviceToHost));
  step("hipMemcpy H2D 8 B (null stream)", hipMemcpy(d, h.data(), 8, hipMemcpyHostToDevice));
  step("hipMemsetAsync 1 MB", hipMemsetAsync(d, 0, 1 << 20, s));
  step("hipStreamSynchronize", hipStreamSynchronize(s));
  k_touch<<<1024, 256>>>(d, 1 << 18);
  step("kernel on the null stream", hipGetLastError());
  step("hipDeviceSynchronize", hipDeviceSynchronize());
  hipStream_t s2;
  step("second stream (same priority)", hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
  k_touch<<<1024, 256, 0, s2>>>(d, 1 << 18);
  step("kernel on the second stream", hipGetLastError());
  step("hipStreamWaitEvent (cross-stream)", hipStreamWaitEvent(s, ev, 0));
  step("hipDeviceSynchronize", hipDeviceSynchronize());
  return 0;
}
