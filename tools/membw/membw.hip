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

// witness-row pattern: grid (chunks per row, rows); row r starts at r * stride bytes
template <int PRO>
__global__ void __launch_bounds__(256) k_write_rows(uint8_t* dst, size_t stride, uint32_t row_elems, uint32_t chunk,
                                                    const uint32_t* src) {
  __shared__ uint32_t core[256];
  if (PRO) {  // a prologue like the emitters': a global load into LDS and a barrier
    core[threadIdx.x] = src[(blockIdx.y * 977u + blockIdx.x * 13u + threadIdx.x) & 0xFFFFF];
    __syncthreads();
  }
  uint32_t s0 = blockIdx.x * chunk;
  uint8_t* row = dst + (size_t)blockIdx.y * stride;
  for (uint32_t q = threadIdx.x; q < chunk && s0 + q < row_elems; q += blockDim.x) {
    uint32_t e = s0 + q;
    u32x4 a = {PRO ? core[q & 255] : e, 0u, 0u, 0u}, b = {0u, 0u, 0u, 0u};
    u32x4* p = reinterpret_cast<u32x4*>(row + 32ull * e);
    p[0] = a; p[1] = b;
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
  {
    // 2048-witness-like rows: stride 72,054,528 B (the canonical witness), 1.66M elements per row
    // written (the SHA share), chunk 4096; rows limited to what fits in the 16 GiB buffer
    const size_t stride = 72054528;
    const uint32_t row_elems = 1688097;  // 54,019,104 B / 32
    const uint32_t rows = (uint32_t)(bytes / stride) - 1;
    const uint32_t chunk = 4096, cpr = (row_elems + chunk - 1) / chunk;
    const double wbytes = (double)rows * row_elems * 32;
    uint32_t* src; hipMalloc(&src, 4u << 20); hipMemset(src, 1, 4u << 20);
    for (int pro = 0; pro < 2; pro++) {
      for (size_t st : {stride, (size_t)row_elems * 32, (stride + 255) / 256 * 256}) {
        hipDeviceSynchronize();
        float best = 1e30f;
        for (int r = 0; r < 5; r++) {
          hipEventRecord(a);
          if (pro) hipLaunchKernelGGL(k_write_rows<1>, dim3(cpr, rows), dim3(256), 0, 0, d, st, row_elems, chunk, src);
          else hipLaunchKernelGGL(k_write_rows<0>, dim3(cpr, rows), dim3(256), 0, 0, d, st, row_elems, chunk, src);
          hipEventRecord(b); hipEventSynchronize(b);
          float ms; hipEventElapsedTime(&ms, a, b); if (ms < best) best = ms;
        }
        printf("rows=%u stride=%zu prologue=%d                %8.1f GB/s  (%.2f ms)\n", rows, st, pro,
               wbytes / best / 1e6, best);
      }
    }
  }
  run("hipMemsetAsync", [&] { hipMemsetAsync(d, 0, bytes, 0); });
  run("read16/lane grid-stride 4096x256", [&] { hipLaunchKernelGGL(k_read, dim3(4096), dim3(256), 0, 0, d, bytes / 16, sink); });
  hipFree(d);
  return 0;
}
