// Device-side definitions shared by the small-k FIA translation units (models.hip,
// score_mf.hip): model traits, top-K order helpers, wave-level reductions, and the
// per-batch kernel arguments.  gfx950 only.
#pragma once

#include <cmath>
#include <cstdint>

#include "common.h"

namespace fia {

// ------------------------------------------------------------------------------------
// model traits
// ------------------------------------------------------------------------------------
template <int K_>
struct MFm {
  static constexpr int K = K_;
  static constexpr int Ds = K + 1;
  static constexpr int D = 2 * Ds;
  static constexpr int SB = 2 * K + 4;          // per-side record: a, xs, bias, xsb, dup_other, pad
                                                // (even: x_s starts 16-B aligned for k_score_mf_mfma)
  static constexpr int R = 4 + 2 * SB;          // header: inv_n, c_q, x.v, r-hat(u,i)
  static constexpr bool ncf = false;
  __device__ static bool decayed(int a) { return a < K; }
  // reference theta order [p_u, q_i, b_u, b_i]
  __device__ static int ref_index(int a) {
    int side = a >= Ds, j = side ? a - Ds : a;
    return j < K ? side * K + j : 2 * K + side;
  }
};

template <int K_>
struct NCFm {
  static constexpr int K = K_;
  static constexpr int H2 = K / 2;
  static constexpr int Ds = 2 * K;
  static constexpr int D = 2 * Ds;
  static constexpr int SB = 2 * K + 1;          // per-side record: x_mlp, W3g * x_gmf, dup_other
  static constexpr int R = 4 + 2 * SB;          // header: inv_n, c_q, x.v, r-hat(u,i)
  static constexpr bool ncf = true;
  __device__ static bool decayed(int) { return true; }
  // reference theta order [Pm_u, Qm_i, Pg_u, Qg_i]
  __device__ static int ref_index(int a) {
    int side = a >= Ds, j = side ? a - Ds : a;
    return j < K ? side * K + j : 2 * K + side * K + (j - K);
  }
};

__device__ __forceinline__ int tri(int r, int c) { return (r * (r + 1)) / 2 + c; }

// Gram cache element (R >= C) of one side block.  Packed lower triangle, except NCF k = 16
// (Ds = 32), kept in the row-pair layout of k_solve_rows: lane t of a side system owns rows t
// and 31 - t, slot C of row t and slot 32 - C of row 31 - t (33 slots per lane), element
// slot * 16 + t -- one slot of the system's 16 lanes is one 128-B line.
template <class M>
__device__ __forceinline__ int gidx(int R, int C) {
  if constexpr (M::ncf && M::Ds == 32) return R < 16 ? C * 16 + R : (32 - C) * 16 + (31 - R);
  else return tri(R, C);
}
template <class M>
constexpr bool pair_layout() { return M::ncf && M::Ds == 32; }
// NCF k <= 16: per list position the Gram pass stores the two ReLU masks of the MLP (bits
// [0, k) z1 > 0, [k, 3k/2) z2 > 0: 4 B) instead of g_mlp (8k B); scoring rebuilds
// d1 = 1[z1 > 0] (W2 (1[z2 > 0] W3m)) from a 2^(k/2)-row LDS table and dots it with
// y = W1_side^T x_mlp (the record's MLP block after k_ncf_rec_y), since
// x_mlp . g_mlp = x_mlp . (W1_side d1) = (W1_side^T x_mlp) . d1
template <class M>
constexpr bool mask_path() { return M::ncf && M::K <= 16; }

// 4 doubles per lane: an f64 MFMA 16x16 tile (C/D layout: element (4 r + (l >> 4), l & 15) in [r])
typedef double d4_t __attribute__((ext_vector_type(4)));

// lane l's double, broadcast to the wave (v_readlane into SGPRs; l compile-time)
__device__ __forceinline__ double readlane_d(double v, int l) {
  const long long b = __double_as_longlong(v);
  const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), l);
  const int hi = __builtin_amdgcn_readlane((int)(b >> 32), l);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}

template <int N>
__device__ __forceinline__ void load_row_f32(const float* __restrict__ src, double* dst) {
  if constexpr (N % 4 == 0) {
    const float4* s4 = reinterpret_cast<const float4*>(src);
#pragma unroll
    for (int c = 0; c < N / 4; ++c) {
      float4 t = s4[c];
      dst[4 * c + 0] = t.x;
      dst[4 * c + 1] = t.y;
      dst[4 * c + 2] = t.z;
      dst[4 * c + 3] = t.w;
    }
  } else {
#pragma unroll
    for (int c = 0; c < N; ++c) dst[c] = src[c];
  }
}

// ------------------------------------------------------------------------------------
// top-K helpers: order = |v| descending, then related position ascending
// ------------------------------------------------------------------------------------
__device__ __forceinline__ double topk_key(double v) {
  double a = fabs(v);
  return (a != a) ? -1.0 : a;     // NaN ranks last among real candidates
}
__device__ __forceinline__ bool better(double a1, int p1, double a2, int p2) {
  return a1 > a2 || (a1 == a2 && p1 < p2);
}

// The best (key, position, value) of the wave, in every lane.  `better` is a strict total
// order on (key, position) -- positions are unique, invalid lanes all carry the same
// (-2, INT_MAX, 0) -- so the result does not depend on the reduction order: DPP row
// rotations inside each 16-lane row, then permlane swaps across the rows (all VALU; the
// ds_bpermute butterfly it replaces waited an LDS round trip per level, six per call)
template <int CTRL>
__device__ __forceinline__ int dpp_i32(int x) {
  // old = x: a disabled source lane returns the lane's own value (a no-op merge)
  return __builtin_amdgcn_update_dpp(x, x, CTRL, 0xf, 0xf, false);
}
__device__ __forceinline__ void best_take(double& a, int& p, double& v, double oa, int op, double ov) {
  if (better(oa, op, a, p)) { a = oa; p = op; v = ov; }
}
template <int CTRL>
__device__ __forceinline__ void best_dpp_step(double& a, int& p, double& v) {
  const long long ab = __double_as_longlong(a), vb = __double_as_longlong(v);
  const int alo = dpp_i32<CTRL>((int)(ab & 0xffffffffll)), ahi = dpp_i32<CTRL>((int)(ab >> 32));
  const int vlo = dpp_i32<CTRL>((int)(vb & 0xffffffffll)), vhi = dpp_i32<CTRL>((int)(vb >> 32));
  const int op = dpp_i32<CTRL>(p);
  best_take(a, p, v, __longlong_as_double(((long long)ahi << 32) | (unsigned)alo), op,
            __longlong_as_double(((long long)vhi << 32) | (unsigned)vlo));
}
// the other row of the lane's pair: rows 0<->1, 2<->3 (SW32 = false) or 0,1<->2,3 (SW32 = true)
template <bool SW32>
__device__ __forceinline__ unsigned other_rows(unsigned x) {
  const bool up = SW32 ? (threadIdx.x & 32) != 0 : (threadIdx.x & 16) != 0;
  if constexpr (SW32) {
    const auto r = __builtin_amdgcn_permlane32_swap(x, x, false, false);   // {[r0 r1 r0 r1], [r2 r3 r2 r3]}
    return up ? r[0] : r[1];
  } else {
    const auto r = __builtin_amdgcn_permlane16_swap(x, x, false, false);   // {[r0 r0 r2 r2], [r1 r1 r3 r3]}
    return up ? r[0] : r[1];
  }
}
template <bool SW32>
__device__ __forceinline__ void best_row_step(double& a, int& p, double& v) {
  const long long ab = __double_as_longlong(a), vb = __double_as_longlong(v);
  const unsigned alo = other_rows<SW32>((unsigned)(ab & 0xffffffffll)), ahi = other_rows<SW32>((unsigned)(ab >> 32));
  const unsigned vlo = other_rows<SW32>((unsigned)(vb & 0xffffffffll)), vhi = other_rows<SW32>((unsigned)(vb >> 32));
  const int op = (int)other_rows<SW32>((unsigned)p);
  best_take(a, p, v, __longlong_as_double(((long long)ahi << 32) | alo), op,
            __longlong_as_double(((long long)vhi << 32) | vlo));
}
__device__ __forceinline__ void wave_best(double& a, int& p, double& v) {
  best_dpp_step<0x128>(a, p, v);   // row_ror:8
  best_dpp_step<0x124>(a, p, v);   // row_ror:4
  best_dpp_step<0x122>(a, p, v);   // row_ror:2
  best_dpp_step<0x121>(a, p, v);   // row_ror:1 -- every lane of a row holds the row's best
  best_row_step<false>(a, p, v);
  best_row_step<true>(a, p, v);
}

// Block-wide K-round selection over per-thread candidate lists (NC each).  Round t
// takes the best candidate strictly worse than round t-1's winner, so no
// "taken" marks are needed (positions are unique).  Writes K (pos, val) pairs.
template <int NC, int NT>
__device__ void block_topk(const double (&ca)[NC], const int (&cp)[NC], const double (&cv)[NC], int K,
                           int32_t* __restrict__ out_pos, double* __restrict__ out_val, double* s_a, int* s_p,
                           double* s_v) {
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
  constexpr int NW = NT / 64;
  double pa = INFINITY;
  int pp = -1;
  for (int t = 0; t < K; ++t) {
    double ba = -2.0, bv = 0.0;
    int bp = 0x7fffffff;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      if (cp[c] >= 0 && better(pa, pp, ca[c], cp[c]) && better(ca[c], cp[c], ba, bp)) {
        ba = ca[c]; bp = cp[c]; bv = cv[c];
      }
    }
    wave_best(ba, bp, bv);
    if (NW > 1) {
      if (lane == 0) { s_a[wave] = ba; s_p[wave] = bp; s_v[wave] = bv; }
      __syncthreads();
      ba = s_a[0]; bp = s_p[0]; bv = s_v[0];
#pragma unroll
      for (int w = 1; w < NW; ++w)
        if (better(s_a[w], s_p[w], ba, bp)) { ba = s_a[w]; bp = s_p[w]; bv = s_v[w]; }
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      bool ok = ba > -1.5;
      out_pos[t] = ok ? bp : -1;
      out_val[t] = ok ? bv : NAN;
    }
    pa = ba; pp = bp;
  }
}

// ------------------------------------------------------------------------------------
// NCF helpers (NCF.py:85-145): z1 = L1_self + L1_other + b1 given; returns r-hat
// pieces via the per-row MLP with the ReLU derivative 1[z > 0] (TF ReluGrad).
// ------------------------------------------------------------------------------------
template <int K>
struct NCFWeights {   // LDS copies (fp64)
  double W2[K * (K / 2)];   // [k][k/2]
  double b2[K / 2];
  double W3[3 * (K / 2)];   // [W3m (k/2) ; W3g (k)]
};

template <int K>
__device__ void load_ncf_weights(NCFWeights<K>& w, const float* W2, const float* b2, const float* W3) {
  constexpr int H = K / 2;
  for (int t = threadIdx.x; t < K * H; t += blockDim.x) w.W2[t] = W2[t];
  for (int t = threadIdx.x; t < H; t += blockDim.x) w.b2[t] = b2[t];
  for (int t = threadIdx.x; t < 3 * H; t += blockDim.x) w.W3[t] = W3[t];
}


__device__ __forceinline__ void wave_lds_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

struct QueryArgs {
  const int32_t* qu;
  const int32_t* qi;
  int64_t U, I;
  const int64_t* ptr[2];
  const int32_t* row[2];
  const int32_t* other[2];
  const float* rating[2];
  const double* gram[2];
  const double* l1[2];
  const float* t[10];
  double wd, damping;
  PairTable pairs;
  // NCF, per list position of each side (written by k_gram_ncf_mfma):
  // g_mlp,j = W1_side . d1_j coordinate-major [k][N], and e_j = r-hat_j - y_j [side][N]
  const double* lgm[2];
  const double* lres;
  int64_t N;
  const double* d1tab;   // NCF k <= 16: d1 table [2^(k/2)][k] (k_ncf_d1_table)
};

}  // namespace fia
