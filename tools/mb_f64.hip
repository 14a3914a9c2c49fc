// Microbenchmark: do f64 MFMA (v_mfma_f64_16x16x4_f64) and f64 VALU (v_fma_f64) run
// concurrently on gfx950?  One 256-thread workgroup per CU (one wave per SIMD) or
// 512 threads (two waves per SIMD), every CU busy.  Modes:
//   0: MFMA only (4 independent accumulators)        1: VALU only (8 independent chains)
//   2: same wave, MFMA + VALU interleaved             3: two waves per SIMD, wave parity picks
//                                                        MFMA or VALU
// Prints kernel time and the implied rates.
//   hipcc --offload-arch=gfx950 -O3 tools/mb_f64.hip -o tools/mb_f64 && tools/mb_f64
#include <hip/hip_runtime.h>
#include <cstdio>

typedef double d4_t __attribute__((ext_vector_type(4)));

template <int MODE>
__global__ void kern(double* out, int iters, double a0, double b0) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  double a = a0 + lane * 1e-3, b = b0 - lane * 1e-3;
  d4_t c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
  double v[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) v[j] = a + j;
  const bool do_m = MODE == 0 || MODE == 2 || (MODE == 3 && (wave & 4) == 0);
  const bool do_v = MODE == 1 || MODE == 2 || (MODE == 3 && (wave & 4) != 0);
  for (int it = 0; it < iters; ++it) {
    if (MODE == 4) {          // one dependent accumulator chain
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c0, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c0, 0, 0, 0);
    } else if (MODE == 5) {   // two chains
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c1, 0, 0, 0);
    } else if (do_m) {
      c0 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c0, 0, 0, 0);
      c1 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, a, c1, 0, 0, 0);
      c2 = __builtin_amdgcn_mfma_f64_16x16x4f64(a, a, c2, 0, 0, 0);
      c3 = __builtin_amdgcn_mfma_f64_16x16x4f64(b, b, c3, 0, 0, 0);
    }
    if (do_v) {
      // 4 MFMAs = 4 x 1024 FMAs = 64 wave-wide FMA instructions of work
#pragma unroll
      for (int r = 0; r < 8; ++r)
#pragma unroll
        for (int j = 0; j < 8; ++j) v[j] = fma(v[j], b, a);
    }
  }
  double s = c0[0] + c1[1] + c2[2] + c3[3];
#pragma unroll
  for (int j = 0; j < 8; ++j) s += v[j];
  if (s == 12345.678) out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

int main() {
  int cus = 0;
  hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0);
  double* out;
  hipMalloc(&out, sizeof(double) * cus * 1024);
  hipEvent_t e0, e1;
  hipEventCreate(&e0);
  hipEventCreate(&e1);
  const int iters = 20000;
  auto run = [&](auto kfn, int threads, const char* name, double mfma_per_wave_it, double valu_per_wave_it) {
    hipLaunchKernelGGL(kfn, dim3(cus), dim3(threads), 0, 0, out, 100, 1.0, 0.5);
    hipDeviceSynchronize();
    hipEventRecord(e0);
    hipLaunchKernelGGL(kfn, dim3(cus), dim3(threads), 0, 0, out, iters, 1.0, 0.5);
    hipEventRecord(e1);
    hipEventSynchronize(e1);
    float ms = 0;
    hipEventElapsedTime(&ms, e0, e1);
    const double waves = (double)cus * threads / 64;
    const double fma = waves * iters * (mfma_per_wave_it * 1024 + valu_per_wave_it * 64);
    printf("%-40s %8.3f ms  %7.2f TFLOP/s f64 (2*FMA)\n", name, ms, 2 * fma / (ms * 1e-3) / 1e12);
  };
  run(kern<0>, 256, "MFMA only, 1 wave/SIMD", 4, 0);
  run(kern<1>, 256, "VALU only, 1 wave/SIMD", 0, 64);
  run(kern<2>, 256, "MFMA+VALU same wave, 1 wave/SIMD", 4, 64);
  run(kern<0>, 512, "MFMA only, 2 waves/SIMD", 4, 0);
  run(kern<1>, 512, "VALU only, 2 waves/SIMD", 0, 64);
  run(kern<3>, 512, "MFMA wave + VALU wave per SIMD", 2, 32);
  run(kern<4>, 256, "MFMA 1 dependent chain, 1 wave/SIMD", 4, 0);
  run(kern<5>, 256, "MFMA 2 chains, 1 wave/SIMD", 4, 0);
  run(kern<4>, 512, "MFMA 1 dependent chain, 2 waves/SIMD", 4, 0);
  return 0;
}
