// MFMA issue-rate probe (profiles only, not in any library): back-to-back
// f16 MFMAs of one shape on random operands, 4 independent accumulators per
// wave, 16 waves per CU; reports ns per MFMA per SIMD and TFLOP/s.
// Shapes: 0 = 32x32x16 f16, 1 = 16x16x32 f16, 2 = 16x16x16 f16, 3 = 32x32x8 f16,
// 4 = 16x16x32 + 16x16x16 pair (the split build's 3-product step on 16x16 tiles),
// 5 = 16x16x32 f16 on 8 accumulators.  argv: iters, workgroups (4 waves) per CU.
// Build: hipcc --offload-arch=gfx950 -O3 -o scripts/mfma_rate <this file>
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>

typedef _Float16 h8 __attribute__((ext_vector_type(8)));
typedef _Float16 h4 __attribute__((ext_vector_type(4)));
typedef float f16v __attribute__((ext_vector_type(16)));
typedef float f4v __attribute__((ext_vector_type(4)));

// Each MFMA is an asm statement on a fixed accumulator ("+v"), so the
// compiler can neither rename the accumulators nor move them between register
// files inside the loop (plain builtins got v_accvgpr moves in the 16x16 loops).
#define MF(INS, ACC, A, B) asm volatile(INS " %0, %1, %2, %0" : "+v"(ACC) : "v"(A), "v"(B))

template <int S>
__global__ __launch_bounds__(256) void rate_kernel(const _Float16* __restrict__ in, float* out, int iters) {
  const int lane = threadIdx.x & 63;
  h8 a, b;
  h4 c, d;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    a[j] = in[(lane * 8 + j) & 1023];
    b[j] = in[(lane * 8 + j + 512) & 1023];
  }
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    c[j] = a[j];
    d[j] = b[j + 4];
  }
  if constexpr (S == 0 || S == 3) {
    f16v acc[4] = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int t = 0; t < 4; ++t) {
        if constexpr (S == 0) MF("v_mfma_f32_32x32x16_f16", acc[t], a, b);
        else MF("v_mfma_f32_32x32x8_f16", acc[t], c, d);
      }
    }
    asm volatile("s_nop 15\n s_nop 15" ::: "memory");
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int r = 0; r < 16; ++r) s += acc[t][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  } else {
    constexpr int NA = S == 5 ? 8 : 4;
    f4v acc[NA] = {};
    for (int i = 0; i < iters; ++i) {
#pragma unroll
      for (int t = 0; t < NA; ++t) {
        if constexpr (S == 1 || S == 5) MF("v_mfma_f32_16x16x32_f16", acc[t], a, b);
        else if constexpr (S == 2) MF("v_mfma_f32_16x16x16_f16", acc[t], c, d);
        else {
          MF("v_mfma_f32_16x16x32_f16", acc[t], a, b);
          MF("v_mfma_f32_16x16x16_f16", acc[t], c, d);
        }
      }
    }
    asm volatile("s_nop 15\n s_nop 15" ::: "memory");
    float s = 0.f;
#pragma unroll
    for (int t = 0; t < NA; ++t)
#pragma unroll
      for (int r = 0; r < 4; ++r) s += acc[t][r];
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
  }
}

int main(int argc, char** argv) {
  const int iters = argc > 1 ? atoi(argv[1]) : 20000;
  hipDeviceProp_t p;
  hipGetDeviceProperties(&p, 0);
  const int per_cu = argc > 2 ? atoi(argv[2]) : 4;
  const int cus = p.multiProcessorCount, blocks = cus * per_cu;
  _Float16* in;
  float* out;
  hipMalloc(&in, 1024 * sizeof(_Float16));
  hipMalloc(&out, (size_t)blocks * 256 * sizeof(float));
  _Float16 h[1024];
  srand(1);
  for (int i = 0; i < 1024; ++i) h[i] = (_Float16)((rand() / (float)RAND_MAX) * 2.f - 1.f);
  hipMemcpy(in, h, sizeof(h), hipMemcpyHostToDevice);
  const char* names[6] = {"32x32x16_f16", "16x16x32_f16", "16x16x16_f16", "32x32x8_f16",
                          "16x16x32+16x16x16", "16x16x32_f16_8acc"};
  const double flops_per[6] = {32. * 32 * 16 * 2, 16. * 16 * 32 * 2, 16. * 16 * 16 * 2,
                               32. * 32 * 8 * 2, 16. * 16 * 48 * 2, 16. * 16 * 32 * 2};
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  for (int round = 0; round < 3; ++round)
    for (int s = 0; s < 6; ++s) {
      auto launch = [&]() {
        switch (s) {
          case 0: rate_kernel<0><<<blocks, 256>>>(in, out, iters); break;
          case 1: rate_kernel<1><<<blocks, 256>>>(in, out, iters); break;
          case 2: rate_kernel<2><<<blocks, 256>>>(in, out, iters); break;
          case 3: rate_kernel<3><<<blocks, 256>>>(in, out, iters); break;
          case 4: rate_kernel<4><<<blocks, 256>>>(in, out, iters); break;
          default: rate_kernel<5><<<blocks, 256>>>(in, out, iters); break;
        }
      };
      launch();
      hipEventRecord(e0);
      launch();
      hipEventRecord(e1);
      hipEventSynchronize(e1);
      float ms = 0.f;
      hipEventElapsedTime(&ms, e0, e1);
      const double n_mfma = (double)blocks * 4 * iters * (s == 5 ? 8 : 4);   // waves x iters x acc
      const double per_simd = n_mfma / (cus * 4.0);
      printf("{\"waves_per_simd\": %d, \"round\": %d, \"shape\": \"%s\", \"ms\": %.3f, \"ns_per_mfma_per_simd\": %.3f, "
             "\"tflops\": %.1f}\n",
             per_cu, round, names[s], ms, ms * 1e6 / per_simd, n_mfma * flops_per[s] / (ms * 1e-3) / 1e12);
    }
  return 0;
}
