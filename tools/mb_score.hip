// Microbenchmark / ablation harness for the scoring kernel's memory pattern
// (not part of the library).  Synthetic data with the ml-1m-ex MF k=16 shape:
// N related ratings in chunks of 256, each row gathers a 64-B embedding row of
// a 3706-row table + a bias, computes two fp64 dots, writes 8 B + 8 B.
//   hipcc --offload-arch=gfx950 -O3 -o mb_score tools/mb_score.hip && ./mb_score
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <random>

#define CK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("HIP %s @%d\n", hipGetErrorString(e), __LINE__); exit(1);} } while (0)

constexpr int K = 16;
constexpr int NREC = 12074;
constexpr int RSZ = 2 * K + 8;

__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

// MODE bits: 1 = gather from row 0 (no randomness), 2 = fp32 math, 4 = no stores,
//            8 = no gathers at all (use list value), 16 = bias folded in padded table,
//            32 = nontemporal stores, 64 = sc1 (agent relaxed atomic) stores,
//            128 = nontemporal list loads, 256 = only the influence store
template <int RW, int MODE>
__global__ __launch_bounds__(256) void k_v0(int64_t nchunks, int64_t N, const int* __restrict__ other,
                                            const float* __restrict__ rating, const int* __restrict__ rowi,
                                            const float* __restrict__ T, const float* __restrict__ bias,
                                            const float* __restrict__ Tp, const double* __restrict__ rec,
                                            double* __restrict__ infl, long long* __restrict__ rel) {
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t ch = (int64_t)blockIdx.x * 4 + wave; ch < nchunks; ch += stride) {
    const int64_t base = ch * 64 * RW;
    const int q = (int)((ch * 2654435761ull) % NREC);
    const double* R = rec + (int64_t)q * RSZ;
    const double rv = R[lane < RSZ ? lane : 0];
    int o_[RW], row_[RW];
    float y_[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int64_t li = base + r * 64 + lane;
      if (MODE & 128) {
        o_[r] = __builtin_nontemporal_load(other + li);
        y_[r] = __builtin_nontemporal_load(rating + li);
        row_[r] = __builtin_nontemporal_load(rowi + li);
      } else {
        o_[r] = other[li];
        y_[r] = rating[li];
        row_[r] = rowi[li];
      }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) asm volatile("" ::"v"(o_[r]), "v"(row_[r]), "v"(y_[r]));
    float4 g[RW][K / 4];
    float gb[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int o = (MODE & 1) ? 0 : o_[r];
      if (MODE & 8) {
#pragma unroll
        for (int c = 0; c < K / 4; ++c) g[r][c] = make_float4(o_[r], c, 1.f, 2.f);
        gb[r] = 0.5f;
      } else if (MODE & 16) {
        const float4* s = reinterpret_cast<const float4*>(Tp + (int64_t)o * 20);
#pragma unroll
        for (int c = 0; c < K / 4; ++c) g[r][c] = s[c];
        gb[r] = Tp[(int64_t)o * 20 + 16];
      } else {
        const float4* s = reinterpret_cast<const float4*>(T + (int64_t)o * K);
#pragma unroll
        for (int c = 0; c < K / 4; ++c) g[r][c] = s[c];
        gb[r] = bias[o];
      }
    }
#pragma unroll
    for (int r = 0; r < RW; ++r) {
#pragma unroll
      for (int c = 0; c < K / 4; ++c) asm volatile("" ::"v"(g[r][c].x), "v"(g[r][c].w));
      asm volatile("" ::"v"(gb[r]));
    }
    double da[RW], dx[RW];
    float fa[RW], fx[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) { da[r] = dx[r] = 0.0; fa[r] = fx[r] = 0.f; }
#pragma unroll
    for (int c4 = 0; c4 < K / 4; ++c4)
#pragma unroll
      for (int cc = 0; cc < 4; ++cc) {
        const double ac = readlane_d(rv, 4 * c4 + cc), xc = readlane_d(rv, K + 4 * c4 + cc);
#pragma unroll
        for (int r = 0; r < RW; ++r) {
          const float t = cc == 0 ? g[r][c4].x : cc == 1 ? g[r][c4].y : cc == 2 ? g[r][c4].z : g[r][c4].w;
          if (MODE & 2) {
            fa[r] = fmaf((float)ac, t, fa[r]);
            fx[r] = fmaf((float)xc, t, fx[r]);
          } else {
            da[r] = fma(ac, (double)t, da[r]);
            dx[r] = fma(xc, (double)t, dx[r]);
          }
        }
      }
    const double b0 = readlane_d(rv, 2 * K), b1 = readlane_d(rv, 2 * K + 1), cq = readlane_d(rv, 2 * K + 2);
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const double e = ((MODE & 2) ? (double)fa[r] : da[r]) + b0 + gb[r] - y_[r];
      const double s = ((MODE & 2) ? (double)fx[r] : dx[r]) + b1;
      const double v = 2.0 * e * s + cq;
      const int64_t li = base + r * 64 + lane;
      if (MODE & 4) {
        asm volatile("" ::"v"(v), "v"(row_[r]));
      } else if (MODE & 32) {
        __builtin_nontemporal_store(v, infl + li);
        if (!(MODE & 256)) __builtin_nontemporal_store((long long)row_[r], rel + li);
      } else if (MODE & 64) {
        __hip_atomic_store(infl + li, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        if (!(MODE & 256)) __hip_atomic_store(rel + li, (long long)row_[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      } else {
        infl[li] = v;
        if (!(MODE & 256)) rel[li] = row_[r];
      }
    }
  }
}

// 4 lanes per row: lane (l & 3) loads float4 #(l&3) of row (l >> 2) of a 16-row group
template <int MODE>
__global__ __launch_bounds__(256) void k_quad(int64_t nchunks, int64_t N, const int* __restrict__ other,
                                              const float* __restrict__ rating, const int* __restrict__ rowi,
                                              const float* __restrict__ T, const float* __restrict__ bias,
                                              const float* __restrict__ Tp, const double* __restrict__ rec,
                                              double* __restrict__ infl, long long* __restrict__ rel) {
  constexpr int RW = 4;
  const int lane = threadIdx.x & 63;
  const int qd = lane & 3, sub = lane >> 2;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t stride = (int64_t)gridDim.x * 4;
  for (int64_t ch = (int64_t)blockIdx.x * 4 + wave; ch < nchunks; ch += stride) {
    const int64_t base = ch * 64 * RW;
    const int q = (int)((ch * 2654435761ull) % NREC);
    const double* R = rec + (int64_t)q * RSZ;
    double a4[4], x4[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) { a4[j] = R[4 * qd + j]; x4[j] = R[K + 4 * qd + j]; }
    const double b0 = R[2 * K], b1 = R[2 * K + 1], cq = R[2 * K + 2];
    int o_[RW], row_[RW];
    float y_[RW];
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      const int64_t li = base + r * 64 + lane;
      o_[r] = other[li];
      y_[r] = rating[li];
      row_[r] = rowi[li];
    }
    // 16 groups of 16 rows: row (16 g + sub) lives in lane (16 g + sub) % 64 of o_[g / 4]
    float4 t[16];
    float gbv[16];
#pragma unroll
    for (int gq = 0; gq < 16; ++gq) {
      const int src = (16 * gq + sub) & 63;
      int o = __shfl(o_[gq / 4], src);
      if (MODE & 1) o = 0;
      if (MODE & 16) {
        t[gq] = reinterpret_cast<const float4*>(Tp + (int64_t)o * 20)[qd];
        gbv[gq] = qd == 0 ? Tp[(int64_t)o * 20 + 16] : 0.f;
      } else {
        t[gq] = reinterpret_cast<const float4*>(T + (int64_t)o * K)[qd];
        gbv[gq] = qd == 0 ? bias[o] : 0.f;
      }
    }
    double res[16];
#pragma unroll
    for (int gq = 0; gq < 16; ++gq) {
      double pa = fma(a4[0], (double)t[gq].x, fma(a4[1], (double)t[gq].y, fma(a4[2], (double)t[gq].z, a4[3] * (double)t[gq].w)));
      double px = fma(x4[0], (double)t[gq].x, fma(x4[1], (double)t[gq].y, fma(x4[2], (double)t[gq].z, x4[3] * (double)t[gq].w)));
      pa += (double)gbv[gq];
      pa += __shfl_xor(pa, 1);
      px += __shfl_xor(px, 1);
      pa += __shfl_xor(pa, 2);
      px += __shfl_xor(px, 2);
      res[gq] = 2.0 * (pa + b0) * (px + b1);
    }
    // back to row-per-lane: row 64 r + lane = group 4 r + lane / 16, sub lane % 16 -> lane 4 (lane % 16)
#pragma unroll
    for (int r = 0; r < RW; ++r) {
      double v = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double w = __shfl(res[4 * r + j], 4 * (lane & 15));
        if ((lane >> 4) == j) v = w;
      }
      v = 2.0 * v - y_[r] + cq;
      const int64_t li = base + r * 64 + lane;
      if (MODE & 4) asm volatile("" ::"v"(v), "v"(row_[r]));
      else { infl[li] = v; rel[li] = row_[r]; }
    }
  }
}

template <class F>
float timeit(F f, int reps) {
  hipEvent_t a, b;
  CK(hipEventCreate(&a)); CK(hipEventCreate(&b));
  f(); f();
  CK(hipDeviceSynchronize());
  CK(hipEventRecord(a));
  for (int i = 0; i < reps; ++i) f();
  CK(hipEventRecord(b));
  CK(hipEventSynchronize(b));
  float ms; CK(hipEventElapsedTime(&ms, a, b));
  return ms / reps;
}

int main() {
  const int I = 3706;
  const int64_t N = 11135975 / 256 * 256;
  std::mt19937 rng(1);
  std::vector<int> other(N), rowi(N);
  std::vector<float> rating(N), T(I * K), bias(I), Tp(I * 20);
  for (int64_t j = 0; j < N; ++j) { other[j] = rng() % I; rowi[j] = rng() % 975460; rating[j] = 1 + rng() % 5; }
  for (auto& v : T) v = (rng() % 1000) / 1000.f;
  for (auto& v : bias) v = (rng() % 1000) / 1000.f;
  for (int i = 0; i < I; ++i) { for (int c = 0; c < K; ++c) Tp[i * 20 + c] = T[i * K + c]; Tp[i * 20 + 16] = bias[i]; }
  std::vector<double> rec(NREC * RSZ);
  for (auto& v : rec) v = (rng() % 1000) / 1000.0;
  int *d_o, *d_r; float *d_y, *d_T, *d_b, *d_Tp; double *d_rec, *d_inf; long long* d_rel;
  CK(hipMalloc(&d_o, N * 4)); CK(hipMalloc(&d_r, N * 4)); CK(hipMalloc(&d_y, N * 4));
  CK(hipMalloc(&d_T, I * K * 4)); CK(hipMalloc(&d_b, I * 4)); CK(hipMalloc(&d_Tp, I * 20 * 4));
  CK(hipMalloc(&d_rec, rec.size() * 8)); CK(hipMalloc(&d_inf, N * 8)); CK(hipMalloc(&d_rel, N * 8));
  CK(hipMemcpy(d_o, other.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_r, rowi.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_y, rating.data(), N * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_T, T.data(), I * K * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_b, bias.data(), I * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_Tp, Tp.data(), I * 20 * 4, hipMemcpyHostToDevice));
  CK(hipMemcpy(d_rec, rec.data(), rec.size() * 8, hipMemcpyHostToDevice));
  const double bytes = N * (12.0 + 16.0);
#define RUN(name, kern, RWv, grid)                                                                                 \
  {                                                                                                                \
    const int64_t nch = N / (64 * RWv);                                                                            \
    float ms = timeit([&] { hipLaunchKernelGGL(kern, dim3(grid), dim3(256), 0, 0, nch, N, d_o, d_y, d_r, d_T, d_b, \
                                               d_Tp, d_rec, d_inf, d_rel); }, 20);                                 \
    printf("%-34s grid %6d  %8.1f us  %6.2f TB/s (28 B/row)\n", name, (int)(grid), ms * 1e3, bytes / (ms * 1e-3) / 1e12); \
  }
  RUN("v0 RW4", (k_v0<4, 0>), 4, 8192);
  RUN("v0 RW4 nt stores", (k_v0<4, 32>), 4, 8192);
  RUN("v0 RW4 gather row0", (k_v0<4, 1>), 4, 8192);
  RUN("v0 RW4 no gathers", (k_v0<4, 8>), 4, 8192);
  RUN("v0 RW4 no stores", (k_v0<4, 4>), 4, 8192);
  RUN("v0 RW4 no gathers no stores", (k_v0<4, 12>), 4, 8192);
  RUN("v0 RW4 fp32 math", (k_v0<4, 2>), 4, 8192);
  RUN("v0 RW4 padded table", (k_v0<4, 16>), 4, 8192);
  RUN("quad", (k_quad<0>), 4, 8192);
  RUN("quad no stores", (k_quad<4>), 4, 8192);
  RUN("quad row0", (k_quad<1>), 4, 8192);
  RUN("v0 RW8 nt stores", (k_v0<8, 32>), 8, 8192);
  RUN("v0 RW2 nt stores", (k_v0<2, 32>), 2, 8192);
  RUN("v0 RW4 nt grid 2048", (k_v0<4, 32>), 4, 2048);
  RUN("v0 RW4 nt grid 32768", (k_v0<4, 32>), 4, 32768);
  return 0;
}
