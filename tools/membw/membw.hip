// Write-bandwidth calibration on MI355X: the witness emitters are write-dominated (32 B per
// signal), so their roofline is the chip's achievable store bandwidth, measured here for the
// store shapes the emitters use. Output: one line per variant, GB/s.
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

typedef uint32_t u32x4 __attribute__((ext_vector_type(4)));

template <int NT, int PER_LANE32>
__global__ void __launch_bounds__(256) k_write(uint8_t* dst, size_t elems, uint32_t chunk) {
  // block b owns elements [b*chunk, (b+1)*chunk) of 32 B each (like an emit work item)
  size_t base = (size_t)blockIdx.x * chunk;
  for (uint32_t q = threadIdx.x; q < chunk; q += blockDim.x) {
    size_t e = base + q;
    if (e >= elems) return;
    u32x4 a = {(uint32_t)e, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
    u32x4* p = reinterpret_cast<u32x4*>(dst + 32 * e);
    if (NT) { __builtin_nontemporal_store(a, p); __builtin_nontemporal_store(b, p + 1); }
    else { p[0] = a; p[1] = b; }
  }
}

// half-wave per element pair: lanes write 16 B each, two lanes per 32-B element (fully contiguous 1 KiB per wave-instruction)
template <int NT>
__global__ void __launch_bounds__(256) k_write16(uint8_t* dst, size_t elems, uint32_t chunk) {
  size_t base = (size_t)blockIdx.x * chunk * 2;
  for (uint32_t q = threadIdx.x; q < 2 * chunk; q += blockDim.x) {
    size_t h = base + q;
    if (h >= 2 * elems) return;
    u32x4 a = {(uint32_t)h, 0u, 0u, 0u};
    u32x4* p = reinterpret_cast<u32x4*>(dst + 16 * h);
    if (NT) __builtin_nontemporal_store(a, p); else p[0] = a;
  }
}

__global__ void k_read(const uint8_t* src, size_t n16, uint32_t* sink) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x, stride = (size_t)gridDim.x * blockDim.x;
  uint32_t acc = 0;
  const u32x4* s = reinterpret_cast<const u32x4*>(src);
  for (; i < n16; i += stride) { u32x4 v = s[i]; acc ^= v.x ^ v.y ^ v.z ^ v.w; }
  if (acc == 0x12345678u) sink[0] = acc;
}

int main() {
  const size_t bytes = 16ull << 30, elems = bytes / 32;
  uint8_t* d; uint32_t* sink;
  if (hipMalloc(&d, bytes) != hipSuccess) { printf("alloc failed\n"); return 1; }
  hipMalloc(&sink, 4);
  hipEvent_t a, b; hipEventCreate(&a); hipEventCreate(&b);
  auto run = [&](const char* name, auto launch) {
    launch(); hipDeviceSynchronize();
    float best = 1e30f;
    for (int r = 0; r < 5; r++) {
      hipEventRecord(a); launch(); hipEventRecord(b); hipEventSynchronize(b);
      float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
    }
    printf("%-40s %8.1f GB/s  (%.2f ms)\n", name, bytes / best / 1e6, best);
  };
  for (uint32_t chunk : {1024u, 4096u}) {
    uint32_t blocks = (uint32_t)((elems + chunk - 1) / chunk);
    char nm[64];
    snprintf(nm, 64, "write32/lane chunk=%u", chunk);
    run(nm, [&] { hipLaunchKernelGGL((k_write<0, 1>), dim3(blocks), dim3(256), 0, 0, d, elems, chunk); });
    snprintf(nm, 64, "write32/lane nt chunk=%u", chunk);
    run(nm, [&] { hipLaunchKernelGGL((k_write<1, 1>), dim3(blocks), dim3(256), 0, 0, d, elems, chunk); });
    snprintf(nm, 64, "write16/lane chunk=%u", chunk);
    run(nm, [&] { hipLaunchKernelGGL((k_write16<0>), dim3(blocks), dim3(256), 0, 0, d, elems, chunk); });
    snprintf(nm, 64, "write16/lane nt chunk=%u", chunk);
    run(nm, [&] { hipLaunchKernelGGL((k_write16<1>), dim3(blocks), dim3(256), 0, 0, d, elems, chunk); });
  }
  run("hipMemsetAsync", [&] { hipMemsetAsync(d, 0, bytes, 0); });
  run("read16/lane grid-stride 4096x256", [&] { hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, d, bytes / 16, sink); });
  hipFree(d);
  return 0;
}
