// Micro-benchmark of the HTTP walk's dependent LDS chain (not product code).
//
//   hipcc -O3 --offload-arch=gfx950 tools/lds_chain_bench.hip -o tools/lds_chain_bench
//   ./tools/lds_chain_bench
//
// Two step forms over the same synthetic slot table (28 KiB image, one
// 1024-thread workgroup per CU, 160 KiB of LDS, as the HTTP kernel):
//   check:  s = (sel >> 16) + b; e = img[s]; sel = label(e) == b ? e : dead
//           (LdsChain::step before: compare, select, add, scale)
//   select: a = label(e) == b_prev ? row_bytes(e) + 4 b : dead_bytes + 4 b;
//           e = img[a]  (rows as LDS byte addresses, 4 b computed off the
//           chain: the compare and the row add side by side, then the select;
//           every address stays inside the table)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CK(x)                                                                          \
  do {                                                                                 \
    hipError_t e_ = (x);                                                               \
    if (e_ != hipSuccess) {                                                            \
      std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
      std::exit(1);                                                                    \
    }                                                                                  \
  } while (0)

constexpr int kBlock = 1024;
constexpr uint32_t kImgWords = 7168;  // 28 KiB
constexpr uint32_t kRows = kImgWords / 256 - 1;
constexpr uint32_t kLdsBytes = 160 * 1024;

typedef __attribute__((address_space(3))) const uint32_t* lds_cptr;

__device__ __forceinline__ uint32_t lds_at(uint32_t byte_addr) {
  return *reinterpret_cast<lds_cptr>(static_cast<uintptr_t>(byte_addr));
}

__device__ __forceinline__ uint32_t mix(uint32_t x) {
  x ^= x >> 16;
  x *= 0x7feb352du;
  x ^= x >> 15;
  x *= 0x846ca68bu;
  x ^= x >> 16;
  return x;
}

// kForm 0: check, 1: select.  Table word i (row r = i / 256 + 1, label i % 256)
// points to a pseudo-random row; every slot's label is its own byte, so no
// walk dies and both forms do identical work.
template <int kForm>
__global__ __launch_bounds__(kBlock) void chain_kernel(const uint32_t* __restrict__ tab, uint32_t steps,
                                                       uint32_t* __restrict__ out, unsigned long long* __restrict__ cyc) {
  extern __shared__ __align__(16) uint32_t smem[];
  for (uint32_t i = threadIdx.x; i < kImgWords; i += kBlock) smem[i] = tab[(kForm ? 1 : 0) * kImgWords + i];
  __syncthreads();
  const uint32_t tid = blockIdx.x * kBlock + threadIdx.x;
  uint32_t seed = mix(tid * 2654435761u + 17u);
  const uint64_t t0 = __builtin_amdgcn_s_memtime();
  uint32_t acc = 0;
  if (kForm == 0) {
    const uint32_t dead = 0;
    uint32_t sel = (256u) << 16;  // row 1
    for (uint32_t k = 0; k < steps; k += 8) {
      const uint32_t w0 = mix(seed + k), w1 = mix(seed + k + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t b = ((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 0xffu;
        uint32_t s = (sel >> 16) + b;
        asm("" : "+v"(s));
        const uint32_t e = smem[s];
        sel = (e & 0xffu) == b ? e : dead;
      }
      acc += sel;
    }
  } else if (kForm == 1) {
    const uint32_t dead = 0;     // byte address of the dead row
    uint32_t e = (256u * 4u) << 16;  // row 1 (byte address), label 0
    uint32_t bprev = 0;
    for (uint32_t k = 0; k < steps; k += 8) {
      const uint32_t w0 = mix(seed + k), w1 = mix(seed + k + 4);
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const uint32_t b = ((j < 4 ? w0 : w1) >> (8 * (j & 3))) & 0xffu;
        uint32_t b4 = 4u * b;
        asm("" : "+v"(b4));  // off the chain
        uint32_t td = dead + b4;
        asm("" : "+v"(td));  // the dead row's slot, off the chain
        uint32_t t = (e >> 16) + b4;
        asm("" : "+v"(t));  // the row add beside the compare, then one select
        const uint32_t a = (e & 0xffu) == bprev ? t : td;
        e = lds_at(a);
        bprev = b;
      }
      acc += e;
    }
  }
  if (kForm == 2) {
    // OOR form: a = row(e) + 4 b with byte 3 = label(e) ^ b_prev (SDWA,
    // other bytes preserved), so a label mismatch addresses past the LDS
    // and reads 0 (the dead row at address 0)
    uint32_t e = (256u * 4u) << 16;  // row 1 (byte address), label 0
    uint32_t wprev = 0;               // packed bytes of the previous block (byte 3 = b_prev of step 0)
    for (uint32_t k = 0; k < steps; k += 8) {
      const uint32_t w0 = mix(seed + k), w1 = mix(seed + k + 4);
#define STEP(W, SEL, P, PSEL)                                                                           \
  {                                                                                                    \
    uint32_t t;                                                                                        \
    asm("v_lshlrev_b32_sdwa %0, 2, %1 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:DWORD src1_sel:" SEL \
        : "=v"(t) : "v"(W));                                                                            \
    asm("v_add_u32_sdwa %0, %1, %0 dst_sel:DWORD dst_unused:UNUSED_PAD src0_sel:WORD_1 src1_sel:DWORD"  \
        : "+v"(t) : "v"(e));                                                                            \
    asm("v_xor_b32_sdwa %0, %1, %2 dst_sel:BYTE_3 dst_unused:UNUSED_PRESERVE src0_sel:BYTE_0 src1_sel:" \
        PSEL : "+v"(t) : "v"(e), "v"(P));                                                               \
    e = lds_at(t);                                                                                     \
  }
      STEP(w0, "BYTE_0", wprev, "BYTE_3")
      STEP(w0, "BYTE_1", w0, "BYTE_0")
      STEP(w0, "BYTE_2", w0, "BYTE_1")
      STEP(w0, "BYTE_3", w0, "BYTE_2")
      STEP(w1, "BYTE_0", w0, "BYTE_3")
      STEP(w1, "BYTE_1", w1, "BYTE_0")
      STEP(w1, "BYTE_2", w1, "BYTE_1")
      STEP(w1, "BYTE_3", w1, "BYTE_2")
#undef STEP
      wprev = w1;
      acc += e;
    }
  }
  const uint64_t t1 = __builtin_amdgcn_s_memtime();
  out[tid] = acc;
  if ((threadIdx.x & 63) == 0) atomicAdd(cyc, static_cast<unsigned long long>(t1 - t0));
}

// Reads LDS words past the allocation (addresses 160 KiB, 2^18, 2^24 + 4):
// the OOR form relies on such reads returning 0.
__global__ void oor_kernel(uint32_t* out) {
  extern __shared__ __align__(16) uint32_t smem[];
  for (uint32_t i = threadIdx.x; i < kLdsBytes / 4; i += blockDim.x) smem[i] = 0xdeadbeefu;
  __syncthreads();
  uint32_t a = threadIdx.x == 0 ? kLdsBytes : threadIdx.x == 1 ? (1u << 18) : threadIdx.x == 2 ? (1u << 24) + 4u : 0u;
  asm volatile("" : "+v"(a));
  out[threadIdx.x] = lds_at(a);
}

int main() {
  int dev = 0, cus = 0, clk = 0;
  CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
  CK(hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev));
  std::vector<uint32_t> tab(2 * kImgWords, 0);
  uint32_t x = 12345;
  for (uint32_t i = 256; i < kImgWords; ++i) {
    x = x * 1664525u + 1013904223u;
    const uint32_t row = 1 + (x >> 8) % kRows, label = i & 255u;
    tab[i] = (row * 256u) << 16 | label;                       // check: word index of the row
    tab[kImgWords + i] = (row * 256u * 4u) << 16 | label;      // select: byte address of the row
  }
  uint32_t *dtab, *dout;
  unsigned long long* dcyc;
  const int grid = cus;
  const size_t nthr = static_cast<size_t>(grid) * kBlock;
  CK(hipMalloc(&dtab, tab.size() * 4));
  CK(hipMalloc(&dout, nthr * 4));
  CK(hipMalloc(&dcyc, 8));
  CK(hipMemcpy(dtab, tab.data(), tab.size() * 4, hipMemcpyHostToDevice));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(chain_kernel<0>), hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(chain_kernel<1>), hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
  const uint32_t steps = 4096;
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  {
    CK(hipFuncSetAttribute(reinterpret_cast<const void*>(oor_kernel), hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
    hipLaunchKernelGGL(oor_kernel, dim3(1), dim3(64), kLdsBytes, 0, dout);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    uint32_t r[4];
    CK(hipMemcpy(r, dout, 16, hipMemcpyDeviceToHost));
    std::printf("oor reads: @160K %08x @2^18 %08x @2^24+4 %08x in-range %08x\n", r[0], r[1], r[2], r[3]);
  }
  CK(hipFuncSetAttribute(reinterpret_cast<const void*>(chain_kernel<2>), hipFuncAttributeMaxDynamicSharedMemorySize, kLdsBytes));
  for (int form = 0; form < 3; ++form) {
    float best = 1e30f;
    unsigned long long cy = 0;
    for (int rep = 0; rep < 5; ++rep) {
      CK(hipMemset(dcyc, 0, 8));
      CK(hipEventRecord(e0, 0));
      if (form == 0)
        hipLaunchKernelGGL(chain_kernel<0>, dim3(grid), dim3(kBlock), kLdsBytes, 0, dtab, steps, dout, dcyc);
      else if (form == 1)
        hipLaunchKernelGGL(chain_kernel<1>, dim3(grid), dim3(kBlock), kLdsBytes, 0, dtab, steps, dout, dcyc);
      else
        hipLaunchKernelGGL(chain_kernel<2>, dim3(grid), dim3(kBlock), kLdsBytes, 0, dtab, steps, dout, dcyc);
      CK(hipGetLastError());
      CK(hipEventRecord(e1, 0));
      CK(hipEventSynchronize(e1));
      float ms = 0;
      CK(hipEventElapsedTime(&ms, e0, e1));
      if (ms < best) best = ms;
      CK(hipMemcpy(&cy, dcyc, 8, hipMemcpyDeviceToHost));
    }
    const double waves = static_cast<double>(grid) * (kBlock / 64);
    std::printf("form %s: %.3f ms, %.1f wave-cycles per step (s_memtime), %.2f ns per step per wave\n",
                form == 2 ? "oor" : form ? "select" : "check", best, static_cast<double>(cy) / waves / steps,
                best * 1e6 / steps);
  }
  std::printf("cus %d clock_khz %d\n", cus, clk);
  return 0;
}
