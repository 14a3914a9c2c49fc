// FIA hot path for MF and NCF on gfx950: entity Gram caches, per-query exact
// solve, flattened influence scoring with chunk-local top-K, top-K merge.
//
// Math (reference citations inline):
//   theta_t per query (u,i), split into a user block and an item block
//     MF  user [p_u (k), b_u]   item [q_i (k), b_i]            Ds = k+1
//     NCF user [Pm_u, Pg_u]     item [Qm_i, Qg_i]              Ds = 2k
//   g_j = d r_j / d theta_t is nonzero only in the user block for j in R_u and
//   only in the item block for j in C_i (both for the (u,i) row itself), so
//     H_t = (2/n) (A_u (+) B_i) + dup correction + wd*M + damping*I
//   with A_u = sum_{j in R_u} g g^T (per user, independent of i) and B_i the
//   item analogue: the rank-1 second-derivative updates (mf:288-308, 324-351)
//   are accumulated ONCE per entity (k_gram) and every query assembles its
//   Hessian from two cached blocks.
//   x = H_t^{-1} v by an exact fp64 LDL^T in LDS (replaces fmin_ncg, mf:419-433).
//   influence_j = x . (2 e_j g_j + wd*M*theta_t) / n (mf:237-246).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <type_traits>

#include "kern.h"

namespace fia {
namespace {

// ------------------------------------------------------------------------------------
// NCF layer-1 halves: L1[0][u] = Pm_u W1[:k], L1[1][i] = Qm_i W1[k:]  (fp64)
// ------------------------------------------------------------------------------------
template <int K>
__global__ void k_ncf_l1(const float* __restrict__ emb, const float* __restrict__ W1, int row_off, int64_t n_ent,
                         double* __restrict__ out) {
  int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (t >= n_ent * K) return;
  int64_t e = t / K;
  int c = (int)(t % K);
  const float* x = emb + e * K;
  double acc = 0.0;
#pragma unroll
  for (int a = 0; a < K; ++a) acc = fma((double)x[a], (double)W1[(row_off + a) * K + c], acc);
  out[t] = acc;
}

// ------------------------------------------------------------------------------------
// Per-query solve: one wave per query.
// ------------------------------------------------------------------------------------
// In-place LDL^T of the packed lower block [lo, hi) followed by L D L^T x = v.
template <int D>
__device__ void ldlt_solve(double* H, double* v, double* d, double* w, int lo, int hi) {
  const int lane = threadIdx.x;
  for (int j = lo; j < hi; ++j) {
    for (int c = lo + lane; c < j; c += kSolveThreads) w[c] = H[tri(j, c)] * d[c];
    __syncthreads();
    for (int r = j + lane; r < hi; r += kSolveThreads) {
      const double* Lr = H + tri(r, 0);
      double t = Lr[j];
      for (int c = lo; c < j; ++c) t = fma(-Lr[c], w[c], t);
      if (r == j) d[j] = t; else H[tri(r, j)] = t;
    }
    __syncthreads();
    const double dj = d[j];
    for (int r = j + 1 + lane; r < hi; r += kSolveThreads) H[tri(r, j)] /= dj;
    __syncthreads();
  }
  for (int j = lo; j < hi; ++j) {
    const double yj = v[j];
    for (int r = j + 1 + lane; r < hi; r += kSolveThreads) v[r] = fma(-H[tri(r, j)], yj, v[r]);
    __syncthreads();
  }
  for (int j = lo + lane; j < hi; j += kSolveThreads) v[j] /= d[j];
  __syncthreads();
  for (int j = hi - 1; j >= lo; --j) {
    const double xj = v[j];
    const double* Lj = H + tri(j, 0);
    for (int c = lo + lane; c < j; c += kSolveThreads) v[c] = fma(-Lj[c], xj, v[c]);
    __syncthreads();
  }
}

__device__ __forceinline__ double wave_sum(double x) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) x += __shfl_xor(x, off);
  return x;
}


// theta_t, v = d r(u,i)/d theta_t (gnn:155, mf:194,201 / ncf:222,229) and r-hat(u,i) of one
// query into the workgroup's LDS arrays th[D] / g[D] (NTH threads cooperate; r-hat is
// valid in the first wave)
template <class M, int NTH>
__device__ double solve_prologue(const QueryArgs& A, int32_t u, int32_t i, double* __restrict__ th,
                                 double* __restrict__ g, double* __restrict__ sh, const NCFWeights<M::ncf ? M::K : 2>& w,
                                 const double* __restrict__ sW1, const double* __restrict__ sb1) {
  constexpr int K = M::K, Ds = M::Ds;
  const int lane = threadIdx.x;
  double rhat_ui = 0.0;
  if constexpr (!M::ncf) {
    const float* P = A.t[0];
    const float* Qt = A.t[1];
    for (int a = lane; a < K; a += NTH) {
      th[a] = P[(int64_t)u * K + a];
      th[Ds + a] = Qt[(int64_t)i * K + a];
      g[a] = Qt[(int64_t)i * K + a];           // user block of v: q_i
      g[Ds + a] = P[(int64_t)u * K + a];       // item block of v: p_u
    }
    if (lane == 0) {
      th[K] = A.t[2][u];
      th[Ds + K] = A.t[3][i];
      g[K] = 1.0;
      g[Ds + K] = 1.0;
    }
    __syncthreads();
    double part = 0.0;
    for (int a = lane; a < K; a += NTH) part += th[a] * th[Ds + a];
    rhat_ui = wave_sum(part) + th[K] + th[Ds + K] + (double)A.t[4][0];
  } else {
    constexpr int H2 = K / 2;
    const float* Pm = A.t[0];
    const float* Qm = A.t[1];
    const float* Pg = A.t[2];
    const float* Qg = A.t[3];
    double* z1 = sh;            // K
    double* d2 = sh + K;        // K/2
    double* d1 = sh + 2 * K;    // K
    for (int a = lane; a < K; a += NTH) {
      th[a] = Pm[(int64_t)u * K + a];
      th[K + a] = Pg[(int64_t)u * K + a];
      th[Ds + a] = Qm[(int64_t)i * K + a];
      th[Ds + K + a] = Qg[(int64_t)i * K + a];
      z1[a] = A.l1[0][(int64_t)u * K + a] + A.l1[1][(int64_t)i * K + a] + sb1[a];
    }
    __syncthreads();
    double mlp_part = 0.0;
    for (int dd2 = lane; dd2 < H2; dd2 += NTH) {
      double z2 = w.b2[dd2];
      for (int c = 0; c < K; ++c) z2 = fma(w.W2[c * H2 + dd2], z1[c] > 0.0 ? z1[c] : 0.0, z2);
      const bool on = z2 > 0.0;
      d2[dd2] = on ? w.W3[dd2] : 0.0;
      mlp_part += on ? w.W3[dd2] * z2 : 0.0;
    }
    double gmf_part = 0.0;
    for (int a = lane; a < K; a += NTH) gmf_part += w.W3[H2 + a] * th[K + a] * th[Ds + K + a];
    rhat_ui = wave_sum(mlp_part + gmf_part) + (double)A.t[9][0];
    __syncthreads();
    for (int c = lane; c < K; c += NTH) {
      double t = 0.0;
      for (int dd2 = 0; dd2 < H2; ++dd2) t = fma(w.W2[c * H2 + dd2], d2[dd2], t);
      d1[c] = z1[c] > 0.0 ? t : 0.0;
    }
    __syncthreads();
    for (int a = lane; a < 2 * K; a += NTH) {
      // rows a < K: W1[:k] (Pm part, user block); rows a >= K: W1[k:] (Qm part, item block)
      double s = 0.0;
      for (int c = 0; c < K; ++c) s = fma(sW1[a * K + c], d1[c], s);
      if (a < K) g[a] = s; else g[Ds + (a - K)] = s;
    }
    for (int a = lane; a < K; a += NTH) {
      g[K + a] = w.W3[H2 + a] * th[Ds + K + a];        // d r/d Pg_u = W3g * Qg_i
      g[Ds + K + a] = w.W3[H2 + a] * th[K + a];        // d r/d Qg_i = W3g * Pg_u
    }
  }
  __syncthreads();
  return rhat_ui;
}

// Record + x_out of one solved query (first wave only, 64 lanes): v = the solution in
// block order [user block (Ds) | item block (Ds)]
template <class M>
__device__ void solve_epilogue(const QueryArgs& A, int64_t q, int32_t u, int32_t i, int64_t n, double rhat_ui,
                               const double* __restrict__ th, const double* __restrict__ g,
                               const double* __restrict__ v, const NCFWeights<M::ncf ? M::K : 2>& w,
                               double* __restrict__ R, double* __restrict__ x_out) {
  constexpr int K = M::K, Ds = M::Ds, D = M::D;
  const int lane = threadIdx.x & 63;
  if (x_out)
    for (int a = lane; a < D; a += kSolveThreads) x_out[q * D + M::ref_index(a)] = v[a];
  double cq = 0.0, xg_user = 0.0, xg_item = 0.0;
  for (int a = lane; a < D; a += kSolveThreads) {
    const int j = a < Ds ? a : a - Ds;
    if (M::decayed(j)) cq += v[a] * th[a];
    if (a < Ds) xg_user += v[a] * g[a]; else xg_item += v[a] * g[a];
  }
  cq = wave_sum(cq) * A.wd;
  xg_user = wave_sum(xg_user);
  xg_item = wave_sum(xg_item);
  // The (u,i) train row itself has g = v, so x.g = x.v and e = r-hat(u,i) - y: both of
  // its copies in rel (user side and item side) get bit-identical influence, as the
  // reference's per-row sess.run gives them (mf:240-246).
  if (lane == 0) {
    R[0] = 1.0 / (double)n;
    R[1] = cq;
    R[2] = xg_user + xg_item;
    R[3] = rhat_ui;
  }
  double* S0 = R + 4;
  double* S1 = R + 4 + M::SB;
  if constexpr (!M::ncf) {
    const double gb = (double)A.t[4][0];
    for (int a = lane; a < K; a += kSolveThreads) {
      S0[a] = th[a];              // p_u
      S0[K + a] = v[a];           // x_pu
      S1[a] = th[Ds + a];         // q_i
      S1[K + a] = v[Ds + a];      // x_qi
    }
    if (lane == 0) {
      S0[2 * K] = th[K] + gb;     S1[2 * K] = th[Ds + K] + gb;
      S0[2 * K + 1] = v[K];       S1[2 * K + 1] = v[Ds + K];
      S0[2 * K + 2] = (double)i;  S1[2 * K + 2] = (double)u;
    }
  } else {
    // x . g_j = x_mlp . g_mlp,j + (W3g * x_gmf) . gmf_other(j)  (k_score_ncf)
    constexpr int H2 = K / 2;
    for (int c = lane; c < K; c += kSolveThreads) {
      S0[c] = v[c];
      S1[c] = v[Ds + c];
      const double w3g = w.W3[H2 + c];
      S0[K + c] = w3g * v[K + c];
      S1[K + c] = w3g * v[Ds + K + c];
    }
    if (lane == 0) {
      S0[2 * K] = (double)i;  S1[2 * K] = (double)u;
    }
  }
}

// One wave per query, the full D x D packed LDL^T: the queries whose test pair is a train row
// (its Hessian couples the user and item blocks; the side-system solves list them in qlist
// {count, q_0, q_1, ...}).
template <class M>
__global__ __launch_bounds__(kSolveThreads, (M::Ds <= 33 ? 2 : 1)) void k_solve(QueryArgs A, int64_t Q, double* __restrict__ rec,
                                                         double* __restrict__ x_out, const int32_t* __restrict__ qlist) {
  constexpr int K = M::K, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2;
  __shared__ double H[D * (D + 1) / 2];
  __shared__ double v[D], g[D], th[D], dd[D], ww[D];
  __shared__ double sh[4 * K + 8];
  // NCF weights staged once per block (fp64), read by every query the block solves
  __shared__ NCFWeights<M::ncf ? K : 2> w;
  __shared__ double sW1[M::ncf ? 2 * K * K : 1];
  __shared__ double sb1[M::ncf ? K : 1];
  if constexpr (M::ncf) {
    load_ncf_weights<K>(w, A.t[6], A.t[7], A.t[8]);
    for (int t = threadIdx.x; t < 2 * K * K; t += blockDim.x) sW1[t] = (double)A.t[4][t];
    for (int t = threadIdx.x; t < K; t += blockDim.x) sb1[t] = (double)A.t[5][t];
  }
  const int64_t nwork = qlist[0];
  for (int64_t wk = blockIdx.x; wk < nwork; wk += gridDim.x) {
  __syncthreads();
  const int64_t q = qlist[1 + wk];
  const int lane = threadIdx.x;
  const int32_t u = A.qu[q], i = A.qi[q];
  double* R = rec + q * M::R;
  const bool ok_id = (u >= 0 && u < A.U && i >= 0 && i < A.I);
  const int64_t ub = ok_id ? A.ptr[0][u] : 0, du = ok_id ? A.ptr[0][u + 1] - ub : 0;
  const int64_t ib = ok_id ? A.ptr[1][i] : 0, di = ok_id ? A.ptr[1][i + 1] - ib : 0;
  const int64_t n = du + di;
  if (n == 0) {
    if (x_out)
      for (int a = lane; a < D; a += kSolveThreads) x_out[q * D + a] = NAN;
    if (lane == 0) R[0] = NAN;
    continue;
  }
  const double s2n = 2.0 / (double)n;

  const double rhat_ui = solve_prologue<M, kSolveThreads>(A, u, i, th, g, sh, w, sW1, sb1);

  // ---- the (u,i) pair among the train rows (pair set built with the index) ----
  double cdup, rsum;
  A.pairs.lookup((unsigned long long)u * (unsigned long long)A.I + (unsigned long long)i, cdup, rsum);
  const bool coupled = cdup > 0.0;
  const double esum = cdup * rhat_ui - rsum;

  // ---- assemble H and solve ----
  const double* Gu = A.gram[0] + (int64_t)u * ((GS + 1) & ~1);
  const double* Gi = A.gram[1] + (int64_t)i * ((GS + 1) & ~1);
  {
    for (int t = lane; t < D * (D + 1) / 2; t += kSolveThreads) {
      int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
      while (tri(r + 1, 0) <= t) ++r;
      while (tri(r, 0) > t) --r;
      const int c = t - tri(r, 0);
      double h = 0.0;
      if (r < Ds) {
        h = s2n * (Gu[gidx<M>(r, c)] + cdup * g[r] * g[c]);
      } else if (c >= Ds) {
        const int rr = r - Ds, cc = c - Ds;
        h = s2n * (Gi[gidx<M>(rr, cc)] + cdup * g[r] * g[c]);
      } else if (coupled) {
        // cross block: item row rr, user col c: 2 (c g_i g_u^T + esum * d2r/dtheta_i dtheta_u)
        const int rr = r - Ds;
        h = s2n * 2.0 * cdup * g[r] * g[c];
        if constexpr (!M::ncf) {
          if (rr == c && c < K) h += s2n * 2.0 * esum;                     // d2 r / dp_u dq_i = I
        } else {
          if (rr == c && c >= K) h += s2n * 2.0 * esum * (double)A.t[8][K / 2 + (c - K)];   // diag(W3g)
        }
      }
      if (r == c) h += (M::decayed(r < Ds ? r : r - Ds) ? A.wd : 0.0) + A.damping;
      H[t] = h;
    }
    for (int a = lane; a < D; a += kSolveThreads) v[a] = g[a];
    __syncthreads();

    if (coupled) {
      ldlt_solve<D>(H, v, dd, ww, 0, D);
    } else {
      ldlt_solve<D>(H, v, dd, ww, 0, Ds);
      ldlt_solve<D>(H, v, dd, ww, Ds, D);
    }
    __syncthreads();
  }

  solve_epilogue<M>(A, q, u, i, n, rhat_ui, th, g, v, w, R, x_out);
  }   // work loop
}

// Scoring records from a GIVEN inverse HVP (fia_query_batch_x: the reference's cached
// <model>-cg-normal_loss-test-[t].npz when force_refresh is False, mf:210-214): one wave per
// query, theta_t / v / r-hat by the solve prologue, x = x_in (reference theta order)
// instead of a solve, then the solve epilogue's record.
template <class M>
__global__ __launch_bounds__(kSolveThreads) void k_record_x(QueryArgs A, int64_t Q, const double* __restrict__ x_in,
                                                            double* __restrict__ rec, double* __restrict__ x_out) {
  constexpr int K = M::K, D = M::D;
  __shared__ double v[D], g[D], th[D];
  __shared__ double sh[4 * K + 8];
  __shared__ NCFWeights<M::ncf ? K : 2> w;
  __shared__ double sW1[M::ncf ? 2 * K * K : 1];
  __shared__ double sb1[M::ncf ? K : 1];
  if constexpr (M::ncf) {
    load_ncf_weights<K>(w, A.t[6], A.t[7], A.t[8]);
    for (int t = threadIdx.x; t < 2 * K * K; t += blockDim.x) sW1[t] = (double)A.t[4][t];
    for (int t = threadIdx.x; t < K; t += blockDim.x) sb1[t] = (double)A.t[5][t];
  }
  for (int64_t q = blockIdx.x; q < Q; q += gridDim.x) {
    __syncthreads();
    const int lane = threadIdx.x;
    const int32_t u = A.qu[q], i = A.qi[q];
    double* R = rec + q * M::R;
    const bool ok_id = (u >= 0 && u < A.U && i >= 0 && i < A.I);
    const int64_t n = ok_id ? (A.ptr[0][u + 1] - A.ptr[0][u]) + (A.ptr[1][i + 1] - A.ptr[1][i]) : 0;
    if (n == 0) {
      if (x_out)
        for (int a = lane; a < D; a += kSolveThreads) x_out[q * D + a] = NAN;
      if (lane == 0) R[0] = NAN;
      continue;
    }
    const double rhat_ui = solve_prologue<M, kSolveThreads>(A, u, i, th, g, sh, w, sW1, sb1);
    for (int a = lane; a < D; a += kSolveThreads) v[a] = x_in[q * D + M::ref_index(a)];
    __syncthreads();
    solve_epilogue<M>(A, q, u, i, n, rhat_ui, th, g, v, w, R, x_out);
  }
}

// ------------------------------------------------------------------------------------
// Side-system solve on 16x16 tiles (NCF, MF k >= 32): one wave per (query, side) system.
//
// The side block H_b (NM x NM after the MF bias is eliminated first as a Schur complement)
// lives in registers as its upper tiles U[p][j] (p <= j) in the f64-MFMA C/D layout: lane
// l = 16 g + c holds rows 4 r + g (r = 0..3) of column c.  In that layout a tile is at once
// the A operand of its transpose and the B operand of itself, so the blocked right-looking
// LDL^T needs no transposes:
//   panel p:  the 16 rows of block p, [S | I | U[p][p+1..] | rhs_p], are eliminated by 16
//             pivot steps (VALU; the pivot row goes through a per-wave LDS slot, the
//             multipliers are the same row read at the lane's own rows -- S is symmetric),
//             giving [D L^T | W = L_pp^-1 | Y_j = D Z_j | y_p]
//   trailing: U[i][j] -= Z_i^T Y_j and rhs_i -= Z_i^T y_p on v_mfma_f64_16x16x4_f64, the
//             right-hand side held in "column layout" (every column of its tile = the
//             vector), so the update of the right-hand side is one more MFMA product
//   back:     x_p = W_p^T (z_p - sum_{i>p} Z_i x_i), z_p = D^-1 y_p: a 16-lane DPP row sum
//             and a 4-row permlane sum per block
// Replaces the one-column-per-lane solve (LDS broadcast of every pivot column to every
// lane: LDS-bound, and 256+256 registers with spills at MF k = 64).
// ------------------------------------------------------------------------------------
template <int CTRL>
__device__ __forceinline__ double dpp_d(double x) {
  const long long b = __double_as_longlong(x);
  const int lo = __builtin_amdgcn_update_dpp(0, (int)(b & 0xffffffffll), CTRL, 0xf, 0xf, false);
  const int hi = __builtin_amdgcn_update_dpp(0, (int)(b >> 32), CTRL, 0xf, 0xf, false);
  return __longlong_as_double(((long long)hi << 32) | (unsigned)lo);
}
// sum over the 16 lanes of each row (quad_perm [1,0,3,2], [2,3,0,1], row_half_mirror,
// row_mirror); every lane of the row gets the bit-identical sum
__device__ __forceinline__ double row_sum16(double x) {
  x += dpp_d<0xB1>(x);
  x += dpp_d<0x4E>(x);
  x += dpp_d<0x141>(x);
  x += dpp_d<0x140>(x);
  return x;
}
// sum over the 4 rows (lanes c, c+16, c+32, c+48); every lane gets the same sum
__device__ __forceinline__ double col_sum4(double x) {
  const long long b = __double_as_longlong(x);
  const unsigned lo = (unsigned)(b & 0xffffffffll), hi = (unsigned)(b >> 32);
  const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
  const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
  const double s = __longlong_as_double(((long long)h16[0] << 32) | l16[0]) +
                   __longlong_as_double(((long long)h16[1] << 32) | l16[1]);   // rows 0+1 | 2+3
  const long long bs = __double_as_longlong(s);
  const unsigned slo = (unsigned)(bs & 0xffffffffll), shi = (unsigned)(bs >> 32);
  const auto l32 = __builtin_amdgcn_permlane32_swap(slo, slo, false, false);
  const auto h32 = __builtin_amdgcn_permlane32_swap(shi, shi, false, false);
  return __longlong_as_double(((long long)h32[0] << 32) | l32[0]) +
         __longlong_as_double(((long long)h32[1] << 32) | l32[1]);
}

// waves per SIMD the tile solve is compiled for (registers: 4 tiles of state per 16 coordinates)
template <class M>
constexpr int col_waves() {
  return M::Ds <= 16 ? 4 : 2;     // N = 32: two 32-row columns per lane (128 VGPRs of matrix)
}

template <class M>
constexpr int tile_waves() {
  return (M::ncf ? M::Ds : M::K) <= 32 ? 3 : 2;
}

__device__ __forceinline__ void pin_d4(d4_t& t) {
  double a = t[0], b = t[1], c = t[2], d = t[3];
  asm volatile("" : "+v"(a), "+v"(b), "+v"(c), "+v"(d));
  t[0] = a; t[1] = b; t[2] = c; t[3] = d;
}

template <int NT>
__device__ constexpr int ut(int p, int j) { return p * NT - (p * (p - 1)) / 2 + (j - p); }

// Raw loads of one side system (issued together, ahead of the query's dependent prologue):
// the upper tiles of the entity's packed lower Gram G (Ds = NM, + 1 with the MF bias), and
// for the MF bias the bias row at the lane's rows (hr) and column (hc) and its diagonal (hb)
template <int NT, bool EXTRA, bool PAIR = false>
__device__ __forceinline__ void tile_load(const double* __restrict__ G, int g, int c, d4_t (&U)[NT * (NT + 1) / 2],
                                          d4_t (&hr)[NT], double (&hc)[NT], double& hb) {
  // PAIR: NCF k = 16's row-pair Gram layout (gidx)
  auto at = [](int R, int C) { return PAIR ? (R < 16 ? C * 16 + R : (32 - C) * 16 + (31 - R)) : (R * (R + 1)) / 2 + C; };
  constexpr int NM = 16 * NT;
  const double* __restrict__ hrow = G + NM * (NM + 1) / 2;   // MF: packed row NM = the bias row
#pragma unroll
  for (int p = 0; p < NT; ++p)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int R = 16 * p + 4 * r + g;
#pragma unroll
      for (int j = p; j < NT; ++j) {
        const int C = 16 * j + c;
        if (j > p) {
          U[ut<NT>(p, j)][r] = G[at(C, R)];
        } else {
          const int hi = R > C ? R : C, lo = R > C ? C : R;
          U[ut<NT>(p, j)][r] = G[at(hi, lo)];
        }
      }
      if constexpr (EXTRA) hr[p][r] = hrow[R];
    }
  if constexpr (EXTRA) {
#pragma unroll
    for (int j = 0; j < NT; ++j) hc[j] = hrow[16 * j + c];
    hb = hrow[NM];
  }
}

// One side system, from the raw loads: H = (2/n) Gram + (wd + damping) I (the MF bias, not
// decayed, eliminated first: H - h h^T / eta, rhs - h gamma / eta), then the blocked
// LDL^T + solves.  Rt: the right-hand side in column layout (raw, [16p + 4r + g]); gam: its
// bias entry.  xs = the solution [Ds] (LDS, written by lanes 0..15), P = this wave's
// pivot-row slots [2][16 * PS] (LDS).
template <int NT, bool EXTRA>
__device__ void tile_factor(int g, int c, d4_t (&U)[NT * (NT + 1) / 2], d4_t (&Rt)[NT], d4_t (&hr)[NT],
                            double (&hc)[NT], double hb, double gam, double s2n, double wd, double damping,
                            double* __restrict__ xs, double* __restrict__ P) {
  constexpr int NM = 16 * NT, PS = (NT + 3) & ~1;
  d4_t W[NT];
  double ieta = 0.0;
  if constexpr (EXTRA) {
    ieta = 1.0 / (s2n * hb + damping);                       // the bias pivot
#pragma unroll
    for (int j = 0; j < NT; ++j) hc[j] *= s2n;
  }
#pragma unroll
  for (int p = 0; p < NT; ++p)
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const int R = 16 * p + 4 * r + g;
      const double h = EXTRA ? s2n * hr[p][r] * ieta : 0.0;
#pragma unroll
      for (int j = p; j < NT; ++j) {
        double v = s2n * U[ut<NT>(p, j)][r];
        if (j == p) v += (R == 16 * j + c) ? wd + damping : 0.0;
        if constexpr (EXTRA) v = fma(-h, hc[j], v);
        U[ut<NT>(p, j)][r] = v;
      }
      if constexpr (EXTRA) Rt[p][r] = fma(-h, gam, Rt[p][r]);
    }
  // ---- factor + forward solve, panel by panel ----
#pragma unroll
  for (int p = 0; p < NT; ++p) {
    d4_t I;
#pragma unroll
    for (int r = 0; r < 4; ++r) I[r] = (4 * r + g == c) ? 1.0 : 0.0;
    double dv[4] = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      double* __restrict__ Pb = P + (k & 1) * (16 * PS);
      const int kr = k >> 2, kg = k & 3;
      // pivot row k of the panel: slot [c][t], t = 0 S, 1 I, 2.. U[p][p+1..], last rhs
      if (g == kg) {
        Pb[c * PS + 0] = U[ut<NT>(p, p)][kr];
        Pb[c * PS + 1] = I[kr];
#pragma unroll
        for (int j = p + 1; j < NT; ++j) Pb[c * PS + 1 + j - p] = U[ut<NT>(p, j)][kr];
        Pb[c * PS + NT - p + 1] = Rt[p][kr];
      }
      wave_lds_sync();
      const double dk = Pb[k * PS];
      double ij = __builtin_amdgcn_rcp(dk);
      ij = fma(ij, fma(-dk, ij, 1.0), ij);
      ij = fma(ij, fma(-dk, ij, 1.0), ij);
      double f[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (4 * r + 3 <= k) {
          f[r] = 0.0;                                  // rows <= k: finished
        } else {
          const double m = Pb[(4 * r + g) * PS] * ij;  // S[k][row] = S[row][k]
          f[r] = (4 * r > k || g > kg) ? m : 0.0;
        }
      }
      double pv[NT + 2];
#pragma unroll
      for (int t = 0; t < NT - p + 2; ++t) pv[t] = Pb[c * PS + t];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        if (4 * r + 3 <= k) continue;
        U[ut<NT>(p, p)][r] = fma(-f[r], pv[0], U[ut<NT>(p, p)][r]);
        I[r] = fma(-f[r], pv[1], I[r]);
#pragma unroll
        for (int j = p + 1; j < NT; ++j) U[ut<NT>(p, j)][r] = fma(-f[r], pv[1 + j - p], U[ut<NT>(p, j)][r]);
        Rt[p][r] = fma(-f[r], pv[NT - p + 1], Rt[p][r]);
      }
      if (g == kg) dv[kr] = ij;                        // 1/d of this lane's row k
      // materialise this step's updates here: hipcc otherwise sinks the FMAs of rows not yet
      // needed as pivots to their first use and keeps every step's multipliers live (spills)
      pin_d4(U[ut<NT>(p, p)]);
      pin_d4(I);
#pragma unroll
      for (int j = p + 1; j < NT; ++j) pin_d4(U[ut<NT>(p, j)]);
      pin_d4(Rt[p]);
      asm volatile("" : "+v"(dv[kr]));
    }
    W[p] = I;
    // trailing update: U[i][j] -= Z_i^T Y_j, rhs_i -= Z_i^T y_p; keep -Z_i for the back solve
#pragma unroll
    for (int i = p + 1; i < NT; ++i) {
      d4_t Zn;
#pragma unroll
      for (int r = 0; r < 4; ++r) Zn[r] = -U[ut<NT>(p, i)][r] * dv[r];
#pragma unroll
      for (int j = i; j < NT; ++j)
#pragma unroll
        for (int kb = 0; kb < 4; ++kb)
          U[ut<NT>(i, j)] = __builtin_amdgcn_mfma_f64_16x16x4f64(Zn[kb], U[ut<NT>(p, j)][kb], U[ut<NT>(i, j)], 0, 0, 0);
#pragma unroll
      for (int kb = 0; kb < 4; ++kb)
        Rt[i] = __builtin_amdgcn_mfma_f64_16x16x4f64(Zn[kb], Rt[p][kb], Rt[i], 0, 0, 0);
      U[ut<NT>(p, i)] = Zn;
    }
#pragma unroll
    for (int r = 0; r < 4; ++r) Rt[p][r] *= dv[r];     // z_p = D^-1 y_p
  }
  // ---- back solve: x_p = W_p^T (z_p - sum_{i>p} Z_i x_i), x in row layout (lane c) ----
  double xr[NT];
#pragma unroll
  for (int p = NT - 1; p >= 0; --p) {
    double pw = 0.0;
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      double w = Rt[p][r];
      if (p + 1 < NT) {
        double s = 0.0;
#pragma unroll
        for (int i = p + 1; i < NT; ++i) s = fma(U[ut<NT>(p, i)][r], xr[i], s);   // (-Z x)[4r+g]
        w += row_sum16(s);
      }
      pw = fma(W[p][r], w, pw);
    }
    xr[p] = col_sum4(pw);
  }
  if constexpr (EXTRA) {                               // the bias: (gamma - h . x) / eta
    double part = 0.0;
#pragma unroll
    for (int j = 0; j < NT; ++j) part = fma(hc[j], xr[j], part);
    part = g == 0 ? part : 0.0;
    const double hx = wave_sum(part);
    if ((threadIdx.x & 63) == 0) xs[NM] = (gam - hx) * ieta;
  }
  if (g == 0) {
#pragma unroll
    for (int p = 0; p < NT; ++p) xs[16 * p + c] = xr[p];
  }
}

// Two waves per query (wave w = side w: user block, item block), persistent over queries;
// NCF weights staged once per workgroup.  Every global load of a query (ids of the next
// query, list pointers, the pair-set probe, both Gram blocks, MF: the right-hand side) is
// issued before its first dependent use, so a query waits on about two memory latencies.
// Queries whose test pair is a train row (coupled blocks) go to `coupled` {count, q...} for
// the full-D k_solve<M, false>.
template <class M>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(tile_waves<M>()))) void k_solve_tile(
    QueryArgs A, int64_t Q, double* __restrict__ rec, double* __restrict__ x_out, int32_t* __restrict__ coupled_out) {
  constexpr int K = M::K, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  constexpr bool EXTRA = !M::ncf;
  constexpr int NM = EXTRA ? K : Ds, NT = NM / 16, PS = (NT + 3) & ~1, NU = NT * (NT + 1) / 2;
  static_assert(NM % 16 == 0 && NT >= 1 && NT <= 4, "tile solve: 16..64 matrix coordinates");
  __shared__ double th[D], g[D], xs[D];
  __shared__ double Pv[2][2 * 16 * PS];
  __shared__ double sh[4 * K + 8];
  __shared__ NCFWeights<M::ncf ? K : 2> w;
  __shared__ double sW1[M::ncf ? 2 * K * K : 1];
  __shared__ double sb1[M::ncf ? K : 1];
  const int wv = threadIdx.x >> 6;
  if constexpr (M::ncf) {
    load_ncf_weights<K>(w, A.t[6], A.t[7], A.t[8]);
    for (int t = threadIdx.x; t < 2 * K * K; t += blockDim.x) sW1[t] = (double)A.t[4][t];
    for (int t = threadIdx.x; t < K; t += blockDim.x) sb1[t] = (double)A.t[5][t];
  }
  int64_t q = blockIdx.x;
  int32_t un = q < Q ? A.qu[q] : 0, in = q < Q ? A.qi[q] : 0;
  for (; q < Q; q += gridDim.x) {
    const int32_t u = un, i = in;
    if (q + gridDim.x < Q) {                           // the next query's ids, in flight
      un = A.qu[q + gridDim.x];
      in = A.qi[q + gridDim.x];
    }
    __syncthreads();                                   // LDS reuse across queries
    int lane = threadIdx.x & 63;                       // opaque per query (no hoisted addresses)
    asm volatile("" : "+v"(lane));
    const int lg = lane >> 4, lc = lane & 15;
    const bool ok_id = (u >= 0 && u < A.U && i >= 0 && i < A.I);
    const int32_t uu = ok_id ? u : 0, ii = ok_id ? i : 0;
    const int64_t pu0 = A.ptr[0][uu], pu1 = A.ptr[0][uu + 1], pi0 = A.ptr[1][ii], pi1 = A.ptr[1][ii + 1];
    const unsigned long long pkey = (unsigned long long)uu * (unsigned long long)A.I + (unsigned long long)ii;
    unsigned long long ph, pk;
    A.pairs.probe_start(pkey, ph, pk);
    const int32_t ent = wv ? ii : uu;
    d4_t U[NU], Rt[NT], hr[NT];
    double hc[NT], hb = 0.0, gam = 0.0;
    // NT <= 2: the Gram loads go out before the prologue (one memory latency per query); at
    // NT >= 3 holding the raw tiles across the prologue spills (MF k=64: 0.42 vs 0.35 ms), so
    // they are issued after it
    constexpr bool EARLY = NT <= 2;
    if constexpr (EARLY) tile_load<NT, EXTRA, pair_layout<M>()>(A.gram[wv] + (int64_t)ent * GSP, lg, lc, U, hr, hc, hb);
    if constexpr (EXTRA) {                             // MF rhs: [other side's embedding ; 1]
      const float* __restrict__ Eo = A.t[wv ? 0 : 1] + (int64_t)(wv ? uu : ii) * K;
#pragma unroll
      for (int p = 0; p < NT; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) Rt[p][r] = (double)Eo[16 * p + 4 * r + lg];
      gam = 1.0;
    }
    const int64_t n = ok_id ? (pu1 - pu0) + (pi1 - pi0) : 0;
    if (n == 0) {
      if (wv == 0) {
        if (x_out)
          for (int a = lane; a < D; a += 64) x_out[q * D + a] = NAN;
        if (lane == 0) rec[q * M::R] = NAN;
      }
      continue;
    }
    const double s2n = 2.0 / (double)n;
    const double rhat_ui = solve_prologue<M, 128>(A, u, i, th, g, sh, w, sW1, sb1);
    if constexpr (!EXTRA) {                            // NCF rhs from the prologue
#pragma unroll
      for (int p = 0; p < NT; ++p)
#pragma unroll
        for (int r = 0; r < 4; ++r) Rt[p][r] = g[wv * Ds + 16 * p + 4 * r + lg];
    }
    double cdup, rsum;
    A.pairs.probe_finish(pkey, ph, pk, cdup, rsum);
    if (cdup > 0.0) {
      if (threadIdx.x == 0) {
        const int slot = atomicAdd(coupled_out, 1);
        coupled_out[1 + slot] = (int32_t)q;
      }
      continue;
    }
    if constexpr (!EARLY) tile_load<NT, EXTRA, pair_layout<M>()>(A.gram[wv] + (int64_t)ent * GSP, lg, lc, U, hr, hc, hb);
    tile_factor<NT, EXTRA>(lg, lc, U, Rt, hr, hc, hb, gam, s2n, A.wd, A.damping, xs + wv * Ds, &Pv[wv][0]);
    __syncthreads();
    if (wv == 0) solve_epilogue<M>(A, q, u, i, n, rhat_ui, th, g, xs, w, rec + q * M::R, x_out);
  }
}

// ------------------------------------------------------------------------------------
// NCF k <= 16 (side blocks of N = 2k <= 32): QW = 32 / k queries per wave.  A side system
// lives in LS = N / 2 lanes (the user block, then the item block, of each query), lane t
// owning columns t and t + LS in registers: a right-looking LDL^T in which step j publishes
// the pivot column through LDS (every lane stores its two entries A[c][j] = col_c[j]) and
// reads it back as uniform-address ds_read_b128 broadcasts, each value feeding TWO FMAs (one
// per owned column: half the LDS traffic per FMA of a column-per-lane layout, which is what
// bounds this solve).  The forward solve rides along; the backward solve broadcasts x_j by
// DPP row_newbcast.  Every global load of a query is issued before its prologue.
// ------------------------------------------------------------------------------------
// sum over the 2 * LS lanes of one query (its two side systems), every lane of it gets the
// same bits: LS = 16 -- a 16-lane row sum, then rows 2h + 1 and 2h; LS = 8 -- a row sum
template <int LS>
__device__ __forceinline__ double sys_sum(double x) {
  x = row_sum16(x);
  if constexpr (LS == 16) {
    const long long b = __double_as_longlong(x);
    const unsigned lo = (unsigned)(b & 0xffffffffll), hi = (unsigned)(b >> 32);
    const auto l16 = __builtin_amdgcn_permlane16_swap(lo, lo, false, false);
    const auto h16 = __builtin_amdgcn_permlane16_swap(hi, hi, false, false);
    x = __longlong_as_double(((long long)h16[0] << 32) | l16[0]) +
        __longlong_as_double(((long long)h16[1] << 32) | l16[1]);
  } else {
    static_assert(LS == 8, "k = 8 or 16");
  }
  return x;
}

template <int N, int J>
__device__ __forceinline__ double bcast_sys(double x, int t) {
  // lane (J % LS) of each LS-lane system; LS = 16: one system per DPP row, LS = 8: two
  constexpr int LS = N / 2;
  if constexpr (LS == 16) {
    return dpp_d<0x150 + (J % 16)>(x);
  } else {
    static_assert(LS == 8, "k = 8 or 16");
    const double lo = dpp_d<0x150 + (J % 8)>(x), hi = dpp_d<0x150 + 8 + (J % 8)>(x);
    return t >= 0 && (threadIdx.x & 8) ? hi : lo;
  }
}

// NCF prologue for QW queries per wave (LQ = 64 / QW lanes per query): theta_t, v and r-hat
// (ncf:102-145, 181-191; gnn:155) into th[h][D] / g[h][D]; rh[h] = r-hat(u,i)
template <class M, int QW>
__device__ void ncf_prologue_multi(const QueryArgs& A, const int32_t* __restrict__ uq, const int32_t* __restrict__ iq,
                                   double (*th)[M::D], double (*g)[M::D], double (*sh)[4 * M::K + 8],
                                   const NCFWeights<M::K>& w, const double* __restrict__ sW1,
                                   const double* __restrict__ sb1, double* __restrict__ rh) {
  constexpr int K = M::K, Ds = M::Ds, H2 = K / 2, LQ = 64 / QW;
  static_assert(2 * K <= LQ, "one lane per g entry");
  const int h = threadIdx.x / LQ, a = threadIdx.x % LQ;
  const int32_t u = uq[h], i = iq[h];
  double* __restrict__ z1 = sh[h];
  double* __restrict__ d2 = sh[h] + K;
  double* __restrict__ d1 = sh[h] + 2 * K;
  if (a < K) {
    th[h][a] = A.t[0][(int64_t)u * K + a];
    th[h][K + a] = A.t[2][(int64_t)u * K + a];
    th[h][Ds + a] = A.t[1][(int64_t)i * K + a];
    th[h][Ds + K + a] = A.t[3][(int64_t)i * K + a];
    z1[a] = A.l1[0][(int64_t)u * K + a] + A.l1[1][(int64_t)i * K + a] + sb1[a];
  }
  wave_lds_sync();
  double part = 0.0;
  if (a < H2) {
    double z2 = w.b2[a];
#pragma unroll
    for (int c = 0; c < K; ++c) z2 = fma(w.W2[c * H2 + a], z1[c] > 0.0 ? z1[c] : 0.0, z2);
    const bool on = z2 > 0.0;
    d2[a] = on ? w.W3[a] : 0.0;
    part = on ? w.W3[a] * z2 : 0.0;
  }
  if (a < K) part += w.W3[H2 + a] * th[h][K + a] * th[h][Ds + K + a];
#pragma unroll
  for (int off = LQ / 2; off > 0; off >>= 1) part += __shfl_xor(part, off);
  if (a == 0) rh[h] = part + (double)A.t[9][0];
  wave_lds_sync();
  if (a < K) {
    double t = 0.0;
#pragma unroll
    for (int dd = 0; dd < H2; ++dd) t = fma(w.W2[a * H2 + dd], d2[dd], t);
    d1[a] = z1[a] > 0.0 ? t : 0.0;
  }
  wave_lds_sync();
  if (a < 2 * K) {
    // rows a < K: W1[:k] (Pm part, user block); rows a >= K: W1[k:] (Qm part, item block)
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < K; ++c) s = fma(sW1[a * K + c], d1[c], s);
    if (a < K) g[h][a] = s; else g[h][Ds + (a - K)] = s;
  }
  if (a < K) {
    g[h][K + a] = w.W3[H2 + a] * th[h][Ds + K + a];        // d r/d Pg_u = W3g * Qg_i
    g[h][Ds + K + a] = w.W3[H2 + a] * th[h][K + a];        // d r/d Qg_i = W3g * Pg_u
  }
  wave_lds_sync();
}

// Pivot slots of one system: [0, N) the pivot column, N y_J, N + 1 1/d_J.  Every lane
// writes its two entries of column J; the owners of row J add y_J and 1/d_J.
template <int N, int J>
__device__ __forceinline__ void ncf2_publish(const double (&c0)[N], const double (&c1)[N], double y0, double y1,
                                             int t, double* __restrict__ Pb) {
  constexpr int LS = N / 2;
  const int ca = t, cb = t + LS;
  Pb[ca] = c0[J];                                  // A[ca][J] = col_ca[J] (symmetric)
  Pb[cb] = c1[J];
  if (ca == J || cb == J) {                        // the diagonal's owner: y_J and 1/d_J
    const double dj = ca == J ? c0[J] : c1[J];
    double ij = __builtin_amdgcn_rcp(dj);
    ij = fma(ij, fma(-dj, ij, 1.0), ij);
    ij = fma(ij, fma(-dj, ij, 1.0), ij);
    Pb[N] = ca == J ? y0 : y1;
    Pb[N + 1] = ij;
  }
}

// Step J, software-pipelined: the pivot data of step J are in LDS; row J + 1 is updated
// first and published (with y_{J+1} and 1/d_{J+1}) before the remaining FMAs of step J, so
// the next step's LDS round trip overlaps them.
template <int N, int J>
__device__ __forceinline__ void ncf2_step(double (&c0)[N], double (&c1)[N], double& y0, double& y1,
                                          double& di0, double& di1, int t, double* __restrict__ P0,
                                          double* __restrict__ P1) {
  constexpr int LS = N / 2;
  const int ca = t, cb = t + LS;
  double* __restrict__ Pb = (J & 1) ? P1 : P0;
  double* __restrict__ Pn = (J & 1) ? P0 : P1;
  wave_lds_sync();
  const double ij = Pb[N + 1], yj = Pb[N];
  if (ca == J) di0 = ij;
  if (cb == J) di1 = ij;
  const double f0 = ca > J ? c0[J] * ij : 0.0;
  const double f1 = cb > J ? c1[J] * ij : 0.0;
  y0 = fma(-f0, yj, y0);
  y1 = fma(-f1, yj, y1);
  if constexpr (J + 1 < N) {
    const double p = Pb[J + 1];
    c0[J + 1] = fma(-p, f0, c0[J + 1]);
    c1[J + 1] = fma(-p, f1, c1[J + 1]);
    ncf2_publish<N, J + 1>(c0, c1, y0, y1, t, Pn);
  }
#pragma unroll
  for (int r = J + 2; r < N; ++r) {
    const double p = Pb[r];
    c0[r] = fma(-p, f0, c0[r]);
    c1[r] = fma(-p, f1, c1[r]);
  }
  if (ca > J) c0[J] = f0;                          // L[ca][J]
  if (cb > J) c1[J] = f1;
  // materialise this step's updates here (hipcc otherwise sinks each row's FMA to the step
  // that first needs it and keeps every step's pivot values live: spills)
#pragma unroll
  for (int r = J; r < N; ++r) asm volatile("" : "+v"(c0[r]), "+v"(c1[r]));
  asm volatile("" : "+v"(y0), "+v"(y1));
}

template <int N, int J>
__device__ __forceinline__ void ncf2_steps(double (&c0)[N], double (&c1)[N], double& y0, double& y1, double& di0,
                                           double& di1, int t, double* __restrict__ P0, double* __restrict__ P1) {
  if constexpr (J < N) {
    ncf2_step<N, J>(c0, c1, y0, y1, di0, di1, t, P0, P1);
    ncf2_steps<N, J + 1>(c0, c1, y0, y1, di0, di1, t, P0, P1);
  }
}

template <int N, int J>
__device__ __forceinline__ void ncf2_back(const double (&c0)[N], const double (&c1)[N], double& y0, double& y1,
                                          double di0, double di1, int t) {
  // L^T x = D^-1 y from the last row: x_J (final in its owner lane) is broadcast to the
  // system's lanes, every lane with a column c < J removes L[J][c] x_J
  if constexpr (J >= 0) {
    constexpr int LS = N / 2;
    const double own = (J < LS) ? y0 : y1;
    const double xj = bcast_sys<N, J>(own, t);
    const int ca = t, cb = t + LS;
    if (ca < J) y0 = fma(-c0[J] * di0, xj, y0);
    if (cb < J) y1 = fma(-c1[J] * di1, xj, y1);
    ncf2_back<N, J - 1>(c0, c1, y0, y1, di0, di1, t);
  }
}

template <class M>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(col_waves<M>()))) void k_solve_col(
    QueryArgs A, int64_t Q, double* __restrict__ rec, double* __restrict__ x_out, int32_t* __restrict__ coupled_out) {
  constexpr int K = M::K, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1, N = Ds;
  constexpr int LS = N / 2, NSYS = 64 / LS, QW = NSYS / 2, PSTR = N + 2;
  static_assert(M::ncf && (N == 16 || N == 32), "NCF k = 8 or 16");
  __shared__ double th[QW][D], g[QW][D], sh[QW][4 * K + 8], rh[QW], s_cd[QW];
  __shared__ int32_t s_u[QW], s_i[QW];
  __shared__ int64_t s_n[QW];
  __shared__ double Pv[2][NSYS * PSTR];
  __shared__ NCFWeights<K> w;
  __shared__ double sW1[2 * K * K];
  __shared__ double sb1[K];
  load_ncf_weights<K>(w, A.t[6], A.t[7], A.t[8]);
  for (int t = threadIdx.x; t < 2 * K * K; t += blockDim.x) sW1[t] = (double)A.t[4][t];
  for (int t = threadIdx.x; t < K; t += blockDim.x) sb1[t] = (double)A.t[5][t];
  const int64_t stride = (int64_t)gridDim.x * QW;
  for (int64_t q0 = (int64_t)blockIdx.x * QW; q0 < Q; q0 += stride) {
    __syncthreads();
    // lane-derived values made opaque per iteration: hoisted out of the loop, the 2N column
    // addresses and lane masks would stay live across it (spills)
    int lane = threadIdx.x;
    asm volatile("" : "+v"(lane));
    const int sys = lane / LS, t = lane % LS, qs = sys >> 1, sd = sys & 1;
    // lane h < QW: query q0 + h -- ids, related count, first pair-set probe
    unsigned long long pk = 0, ph = 0, pv = 0;
    if (lane < QW) {
      const int64_t q = q0 + lane;
      const int32_t u = q < Q ? A.qu[q] : -1, i = q < Q ? A.qi[q] : -1;
      const bool ok = u >= 0 && u < A.U && i >= 0 && i < A.I;
      const int32_t uu = ok ? u : 0, ii = ok ? i : 0;
      const int64_t nn = ok ? (A.ptr[0][uu + 1] - A.ptr[0][uu]) + (A.ptr[1][ii + 1] - A.ptr[1][ii]) : 0;
      pk = (unsigned long long)uu * (unsigned long long)A.I + (unsigned long long)ii;
      A.pairs.probe_start(pk, ph, pv);
      s_u[lane] = uu;                                // clamped ids (n = 0 for invalid ones)
      s_i[lane] = ii;
      s_n[lane] = nn;
    }
    wave_lds_sync();
    const int32_t ent = sd ? s_i[qs] : s_u[qs];
    const double* __restrict__ Gb = A.gram[sd] + (int64_t)ent * GSP;
    const int ca = t, cb = t + LS;
    // the prologue first: holding the 2N loaded columns across it spills
    ncf_prologue_multi<M, QW>(A, s_u, s_i, th, g, sh, w, sW1, sb1, rh);
    double c0[N], c1[N];
#pragma unroll
    for (int r = 0; r < N; ++r) {
      const int h0 = r > ca ? r : ca, l0 = r > ca ? ca : r;
      const int h1 = r > cb ? r : cb, l1 = r > cb ? cb : r;
      c0[r] = Gb[gidx<M>(h0, l0)];
      c1[r] = Gb[gidx<M>(h1, l1)];
    }
    const int64_t n = s_n[qs];
    // H_b = (2/n) Gram_b + (wd + damping) I  (every NCF coordinate is decayed); n = 0: the
    // system is garbage and its query writes NaN below
    const double s2n = n > 0 ? 2.0 / (double)n : 0.0;
#pragma unroll
    for (int r = 0; r < N; ++r) {
      c0[r] *= s2n;
      c1[r] *= s2n;
    }
#pragma unroll
    for (int r = 0; r < N; ++r) {
      if (r == ca) c0[r] += A.wd + A.damping;
      if (r == cb) c1[r] += A.wd + A.damping;
    }
    double y0 = g[qs][sd * N + ca], y1 = g[qs][sd * N + cb];
    const double g0 = y0, g1 = y1;
    ncf2_publish<N, 0>(c0, c1, y0, y1, t, &Pv[0][sys * PSTR]);
    double di0 = 0.0, di1 = 0.0;
    ncf2_steps<N, 0>(c0, c1, y0, y1, di0, di1, t, &Pv[0][sys * PSTR], &Pv[1][sys * PSTR]);
    y0 *= di0;
    y1 *= di1;
    ncf2_back<N, N - 1>(c0, c1, y0, y1, di0, di1, t);
    if (lane < QW) {                                 // is the test pair a train row?
      double cdup, rsum;
      A.pairs.probe_finish(pk, ph, pv, cdup, rsum);
      s_cd[lane] = cdup;
    }
    wave_lds_sync();
    // ---- record + x_out, lane-parallel: this lane holds x at coordinates ca, cb of side sd
    // of query qs (record layout: solve_epilogue) ----
    {
      const int64_t q = q0 + qs;
      const int64_t nn = s_n[qs];
      const bool live_q = q < Q && nn > 0 && !(s_cd[qs] > 0.0);
      constexpr int H2 = K / 2;
      // x . theta over the decayed coordinates (all of NCF's) and x . v, summed over the query's
      // two systems (2 LS lanes)
      double cq = fma(y0, th[qs][sd * N + ca], y1 * th[qs][sd * N + cb]);
      double xv = fma(y0, g0, y1 * g1);
      cq = sys_sum<LS>(cq);
      xv = sys_sum<LS>(xv);
      if (live_q) {
        double* __restrict__ R = rec + q * M::R;
        double* __restrict__ S = R + 4 + sd * M::SB;
        if (sd == 0 && t == 0) {
          R[0] = 1.0 / (double)nn;
          R[1] = cq * A.wd;
          R[2] = xv;
          R[3] = rh[qs];
        }
        // block coordinates: [0, K) mlp, [K, 2K) gmf; the record holds x_mlp and W3g * x_gmf
        S[ca] = ca < K ? y0 : w.W3[H2 + ca - K] * y0;
        S[cb] = cb < K ? y1 : w.W3[H2 + cb - K] * y1;
        if (t == 0) S[2 * K] = (double)(sd ? s_u[qs] : s_i[qs]);
        if (x_out) {
          x_out[q * D + M::ref_index(sd * Ds + ca)] = y0;
          x_out[q * D + M::ref_index(sd * Ds + cb)] = y1;
        }
      } else if (q < Q && nn == 0) {
        if (x_out) {
          x_out[q * D + sd * Ds + ca] = NAN;
          x_out[q * D + sd * Ds + cb] = NAN;
        }
        if (sd == 0 && t == 0) rec[q * M::R] = NAN;
      } else if (q < Q && sd == 0 && t == 0) {      // coupled: the full-D solve finishes it
        const int slot = atomicAdd(coupled_out, 1);
        coupled_out[1 + slot] = (int32_t)q;
      }
    }
  }
}

// ------------------------------------------------------------------------------------
// NCF k = 16 side-system solve by rows (the default for NCF k = 16), two launches:
//  k_ncf_query_pro: one THREAD per query -- n, the pair-set lookup, r-hat(u,i) and
//    v = d r-hat / d theta_t in block order (ncf:102-145, 181-191; gnn:155) into
//    qpro[q] = {v[D] | r-hat, n, c_dup, 0}.  The MLP is ~0.8 k FMAs per query; computed
//    wave-cooperatively inside the solve (k_solve_col) it took a fifth of that kernel
//    (LDS round trips between tiny loops, by s_memtime stamps of a diagnostic build).
//  k_solve_rows: 16 lanes per side system (4 systems = 2 queries per wave); lane t owns rows
//    t and 31 - t of the lower triangle, 33 entries, loaded from the Gram's row-pair layout
//    (gidx: one 128-B line per slot and system).  Right-looking LDL^T: step J publishes the
//    pivot column through LDS and every lane updates its two rows; a row's entries live in
//    a[16] (row t) / b[32] (row 31 - t), slots past a row's end are scratch, so no FMA needs
//    a mask -- 616 FMAs per lane for the 4 systems (the column layout's full-column updates:
//    992) at 96 VGPRs of matrix instead of 128 + spills.  Column J + 1 is updated and
//    published before the rest of step J, so the LDS round trip overlaps those FMAs; the
//    forward solve rides along, the backward solve is one 16-lane DPP sum per row.
// ------------------------------------------------------------------------------------
template <class M>
constexpr int qpro_stride() { return M::D + 4; }
constexpr int kRowsRG = 8;         // pivot reads per group
constexpr int kRowsWaves = 2;      // 198 VGPRs, no spills; at 3 waves (168 VGPRs) 34 spill: 0.252 vs 0.220 ms at yelp-ex

template <class M>
__global__ __launch_bounds__(256) void k_ncf_query_pro(QueryArgs A, int64_t Q, double* __restrict__ qpro) {
  constexpr int K = M::K, H2 = K / 2, Ds = M::Ds, D = M::D, PS = qpro_stride<M>();
  constexpr int EPL = H2 / 4, GPL = 2 * K / 4, FPL = K / 4;   // per-lane shares of a query's outputs
  static_assert(H2 % 4 == 0, "k a multiple of 8");
  // the MLP weights as fp64 in LDS, read per use as broadcasts (per-use scalar loads of the
  // fp32 tables expose a memory latency per weight)
  __shared__ double sW1[2 * K * K], sW2[K * H2], sW3[3 * H2], sb1[K], sb2[H2];
  for (int e = threadIdx.x; e < 2 * K * K; e += 256) sW1[e] = (double)A.t[4][e];
  for (int e = threadIdx.x; e < K * H2; e += 256) sW2[e] = (double)A.t[6][e];
  for (int e = threadIdx.x; e < 3 * H2; e += 256) sW3[e] = (double)A.t[8][e];
  for (int e = threadIdx.x; e < K; e += 256) sb1[e] = (double)A.t[5][e];
  for (int e = threadIdx.x; e < H2; e += 256) sb2[e] = (double)A.t[7][e];
  __syncthreads();
  // four lanes per query (quad sub = 0..3): each computes a quarter of z2 / g / the gmf terms;
  // every lane of a quad stays active for the quad exchanges
  const int sub = threadIdx.x & 3, base = threadIdx.x & 63 & ~3;
  const int64_t q0 = (int64_t)blockIdx.x * 64 + (threadIdx.x >> 2);
  const bool qok = q0 < Q;
  const int64_t q = qok ? q0 : Q - 1;
  const int32_t u = A.qu[q], i = A.qi[q];
  const bool ok = u >= 0 && u < A.U && i >= 0 && i < A.I;
  const int32_t uu = ok ? u : 0, ii = ok ? i : 0;         // clamped ids (n = 0 for invalid ones)
  const double* __restrict__ l1u = A.l1[0] + (int64_t)uu * K;
  const double* __restrict__ l1i = A.l1[1] + (int64_t)ii * K;
  double z1[K];
#pragma unroll
  for (int a = 0; a < K; ++a) z1[a] = l1u[a] + l1i[a] + sb1[a];
  double d2o[EPL], part = 0.0;
#pragma unroll
  for (int m = 0; m < EPL; ++m) {                 // hidden unit e = m * 4 + sub
    const int e = m * 4 + sub;
    double z2 = sb2[e];
#pragma unroll
    for (int c = 0; c < K; ++c) z2 = fma(sW2[c * H2 + e], z1[c] > 0.0 ? z1[c] : 0.0, z2);
    const bool on = z2 > 0.0;
    d2o[m] = on ? sW3[e] : 0.0;
    part += on ? sW3[e] * z2 : 0.0;
  }
  double d2[H2];
#pragma unroll
  for (int e = 0; e < H2; ++e) d2[e] = __shfl(d2o[e / 4], base + (e & 3));
  double* __restrict__ P = qpro + q * PS;
  const float* __restrict__ pg = A.t[2] + (int64_t)uu * K;
  const float* __restrict__ qg = A.t[3] + (int64_t)ii * K;
#pragma unroll
  for (int m = 0; m < FPL; ++m) {
    const int a = m * 4 + sub;
    const double w3g = sW3[H2 + a], pga = (double)pg[a], qga = (double)qg[a];
    part += w3g * pga * qga;
    if (qok) {
      P[K + a] = w3g * qga;            // d r / d Pg_u = W3g * Qg_i
      P[Ds + K + a] = w3g * pga;       // d r / d Qg_i = W3g * Pg_u
    }
  }
  double d1[K];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    double s = 0.0;
#pragma unroll
    for (int e = 0; e < H2; ++e) s = fma(sW2[c * H2 + e], d2[e], s);
    d1[c] = z1[c] > 0.0 ? s : 0.0;
  }
#pragma unroll
  for (int m = 0; m < GPL; ++m) {      // rows a < K: W1[:k] (user block), a >= K: W1[k:] (item block)
    const int a = m * 4 + sub;
    double s = 0.0;
#pragma unroll
    for (int c = 0; c < K; ++c) s = fma(sW1[a * K + c], d1[c], s);
    if (qok) P[a < K ? a : Ds + (a - K)] = s;
  }
  part += __shfl_xor(part, 1);
  part += __shfl_xor(part, 2);
  if (sub == 0 && qok) {
    const int64_t n = ok ? (A.ptr[0][uu + 1] - A.ptr[0][uu]) + (A.ptr[1][ii + 1] - A.ptr[1][ii]) : 0;
    double cdup, rsum;
    A.pairs.lookup((unsigned long long)uu * (unsigned long long)A.I + (unsigned long long)ii, cdup, rsum);
    P[D] = part + (double)A.t[9][0];
    P[D + 1] = (double)n;
    P[D + 2] = cdup;
    P[D + 3] = 0.0;
  }
}

// Step J of k_solve_rows.  P0 / P1: the pivot slots of even / odd steps ([0, 32) the
// column's rows, 32 y_J); lt / lb: the multipliers of rows t / 31 - t (0 unless the row is
// strictly below the pivot, so finished rows and the pivot row take no update).
template <int J>
__device__ __forceinline__ void rows_step(double (&a)[16], double (&b)[32], double& yt, double& yb, double& dit,
                                          double& dib, int t, double* __restrict__ P0, double* __restrict__ P1) {
  const double* __restrict__ Pb = (J & 1) ? P1 : P0;
  double* __restrict__ Pn = (J & 1) ? P0 : P1;
  const int tb = 31 - t;
  wave_lds_sync();
  const double dj = Pb[J], yj = Pb[32];
  double ij = __builtin_amdgcn_rcp(dj);            // 1/d_J: v_rcp_f64 + two Newton steps
  ij = fma(ij, fma(-dj, ij, 1.0), ij);
  ij = fma(ij, fma(-dj, ij, 1.0), ij);
  double lt = 0.0;
  if constexpr (J < 16) lt = t > J ? a[J] * ij : 0.0;
  const double lb = tb > J ? b[J] * ij : 0.0;
  if (t == J) dit = ij;
  if (tb == J) dib = ij;
  yt = fma(-lt, yj, yt);
  yb = fma(-lb, yj, yb);
  if constexpr (J + 1 < 32) {
    // column J + 1 first, then published for step J + 1 (with y_{J+1} by its owner)
    const double p = Pb[J + 1];
    if constexpr (J + 1 < 16) {
      a[J + 1] = fma(-lt, p, a[J + 1]);
      Pn[t] = a[J + 1];
    }
    b[J + 1] = fma(-lb, p, b[J + 1]);
    Pn[tb] = b[J + 1];
    if constexpr (J + 1 < 16) {
      if (t == J + 1) Pn[32] = yt;
    } else {
      if (tb == J + 1) Pn[32] = yb;
    }
  }
  // the pivot reads in groups of RG columns (a compiler barrier between groups): all of a
  // step's reads hoisted together hold 62 more VGPRs
#pragma unroll
  for (int c = J + 2; c < 16; ++c) {
    if ((c - J - 2) % kRowsRG == kRowsRG - 1) asm volatile("" ::: "memory");
    const double p = Pb[c];
    a[c] = fma(-lt, p, a[c]);
    b[c] = fma(-lb, p, b[c]);
  }
#pragma unroll
  for (int c = (J + 2 > 16 ? J + 2 : 16); c < 32; ++c) {
    if ((c - J - 2) % kRowsRG == kRowsRG - 1) asm volatile("" ::: "memory");
    b[c] = fma(-lb, Pb[c], b[c]);
  }
  if constexpr (J < 16) a[J] = lt;                 // L[t][J], L[31 - t][J]
  b[J] = lb;
  // materialise this step's updates here (hipcc otherwise sinks each row's FMA to the step
  // that first needs it and keeps every step's multipliers live: spills)
#pragma unroll
  for (int c = (J < 16 ? J : 16); c < 16; ++c) asm volatile("" : "+v"(a[c]));
#pragma unroll
  for (int c = J; c < 32; ++c) asm volatile("" : "+v"(b[c]));
  asm volatile("" : "+v"(yt), "+v"(yb));
}

template <int J>
__device__ __forceinline__ void rows_steps(double (&a)[16], double (&b)[32], double& yt, double& yb, double& dit,
                                           double& dib, int t, double* __restrict__ P0, double* __restrict__ P1) {
  if constexpr (J < 32) {
    rows_step<J>(a, b, yt, yb, dit, dib, t, P0, P1);
    rows_steps<J + 1>(a, b, yt, yb, dit, dib, t, P0, P1);
  }
}

// L^T x = z from the last row: x_J = z_J - sum_{r > J} L[r][J] x_r, the sum over the system's
// 16 lanes (each holds L[t][J] x_t + L[31-t][J] x_{31-t}; 0 for rows not below J)
template <int J>
__device__ __forceinline__ void rows_back(const double (&a)[16], const double (&b)[32], double zt, double zb,
                                          double& xt, double& xb, int t) {
  if constexpr (J >= 0) {
    double s = b[J] * xb;
    if constexpr (J < 16) s = fma(a[J], xt, s);
    s = row_sum16(s);
    if constexpr (J < 16) {
      if (t == J) xt = zt - s;
    } else {
      if (31 - t == J) xb = zb - s;
    }
    rows_back<J - 1>(a, b, zt, zb, xt, xb, t);
  }
}

template <class M>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(kRowsWaves))) void k_solve_rows(
    QueryArgs A, int64_t Q, const double* __restrict__ qpro, double* __restrict__ rec, double* __restrict__ x_out,
    int32_t* __restrict__ coupled_out) {
  static_assert(pair_layout<M>(), "NCF k = 16 (side blocks of 32)");
  constexpr int K = M::K, H2 = K / 2, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  constexpr int PS = qpro_stride<M>(), PST = 36;   // 36 doubles: the 4 systems' slots in distinct banks
  __shared__ double Pv[2][4 * PST];
  const int lane = threadIdx.x, sys = lane >> 4, t = lane & 15, h = sys >> 1, sd = sys & 1, tb = 31 - t;
  const int64_t q = (int64_t)blockIdx.x * 2 + h;
  const bool qok = q < Q;
  const int64_t qc = qok ? q : Q - 1;
  const int32_t u = A.qu[qc], i = A.qi[qc];
  const bool okid = u >= 0 && u < A.U && i >= 0 && i < A.I;
  const int32_t uu = okid ? u : 0, ii = okid ? i : 0;
  const int32_t ent = sd ? ii : uu;
  const double* __restrict__ Gb = A.gram[sd] + (int64_t)ent * GSP + t;
  const double* __restrict__ P = qpro + qc * PS;
  double a[16], b[32];
#pragma unroll
  for (int s = 0; s <= 32; ++s) {                 // slot s: row t col s | row 31 - t col 32 - s
    const double v = Gb[s * 16];
    if (s < 16) a[s] = v;
    if (s >= 1) b[32 - s] = v;
  }
  const double nd = P[D + 1];
  // H_b = (2/n) Gram_b + (wd + damping) I  (every NCF coordinate is decayed); n = 0: the
  // system is garbage and its query writes NaN below
  const double s2n = nd > 0.0 ? 2.0 / nd : 0.0;
  const double lam = A.wd + A.damping;
#pragma unroll
  for (int c = 0; c < 16; ++c) a[c] *= s2n;
#pragma unroll
  for (int c = 0; c < 32; ++c) b[c] *= s2n;
#pragma unroll
  for (int c = 0; c < 16; ++c)
    if (c == t) a[c] += lam;
#pragma unroll
  for (int c = 16; c < 32; ++c)
    if (c == tb) b[c] += lam;
  double yt = P[sd * Ds + t], yb = P[sd * Ds + tb], dit = 0.0, dib = 0.0;
  double* __restrict__ P0 = &Pv[0][sys * PST];
  double* __restrict__ P1 = &Pv[1][sys * PST];
  P0[t] = a[0];
  P0[tb] = b[0];
  if (t == 0) P0[32] = yt;
  rows_steps<0>(a, b, yt, yb, dit, dib, t, P0, P1);
  const double zt = yt * dit, zb = yb * dib;
  double xt = 0.0, xb = 0.0;
  rows_back<31>(a, b, zt, zb, xt, xb, t);
  // ---- record + x_out (record layout: solve_epilogue); sums over the query's 2 systems ----
  // (loaded here, not held across the factorization)
  const double rh = P[D], cdup = P[D + 2];
  const double gt = P[sd * Ds + t], gbv = P[sd * Ds + tb];
  // theta at the lane's two coordinates: side 0 [Pm_u | Pg_u], side 1 [Qm_i | Qg_i]
  const double tht = (double)A.t[sd][(int64_t)ent * K + t];
  const double thb = (double)A.t[2 + sd][(int64_t)ent * K + (tb - K)];
  const double w3b = (double)A.t[8][H2 + (tb - K)];
  double cq = fma(xt, tht, xb * thb);
  double xv = fma(xt, gt, xb * gbv);
  cq = sys_sum<16>(cq);
  xv = sys_sum<16>(xv);
  const int64_t n = (int64_t)nd;
  if (qok && n > 0 && !(cdup > 0.0)) {
    double* __restrict__ R = rec + q * M::R;
    double* __restrict__ S = R + 4 + sd * M::SB;
    if (sd == 0 && t == 0) {
      R[0] = 1.0 / nd;
      R[1] = cq * A.wd;
      R[2] = xv;
      R[3] = rh;
    }
    S[t] = xt;                                     // x_mlp
    S[tb] = w3b * xb;                              // W3g * x_gmf
    if (t == 0) S[2 * K] = (double)(sd ? uu : ii);
    if (x_out) {
      x_out[q * D + M::ref_index(sd * Ds + t)] = xt;
      x_out[q * D + M::ref_index(sd * Ds + tb)] = xb;
    }
  } else if (qok && n == 0) {
    if (x_out) {
      x_out[q * D + sd * Ds + t] = NAN;
      x_out[q * D + sd * Ds + tb] = NAN;
    }
    if (sd == 0 && t == 0) rec[q * M::R] = NAN;
  } else if (qok && sd == 0 && t == 0) {          // coupled: the full-D solve finishes it
    const int slot = atomicAdd(coupled_out, 1);
    coupled_out[1 + slot] = (int32_t)q;
  }
}

// ------------------------------------------------------------------------------------
// MF, k = 16 (the headline): a quad of lanes per side system, 16 systems (8 queries) per wave.
// Lane j of a quad owns rows j, j + 4, j + 8, j + 12 of the block's embedding coordinates
// (slot s = row 4 s + j: a[s][c] = H[r][c] for c <= r), their bias-row entries hb[s] =
// H[16][r] and right-hand sides y[s] = v_r; the bias pivot H[16][16] (and y_16) is kept by
// every lane of the quad and eliminated last.  Right-looking LDL^T: step J broadcasts the
// pivot column inside the quad by DPP quad_perm (no LDS), every lane updates its rows; the
// back solve sums each row's terms by two quad DPP steps.  A thread per system (k_solve_tps,
// k = 8) held the whole 17 x 17 block in one lane: at k = 16 that was 256 VGPRs with AGPR
// spills, 378 waves for 12 k queries (one per SIMD), every dependent step exposed.
// ------------------------------------------------------------------------------------
// every lane of the quad gets lane L's value (DPP quad_perm [L, L, L, L])
template <int L>
__device__ __forceinline__ double quad_bcast(double x) {
  return dpp_d<(L | (L << 2) | (L << 4) | (L << 6))>(x);
}
__device__ __forceinline__ double quad_sum(double x) {
  x += dpp_d<0xB1>(x);      // quad_perm [1, 0, 3, 2]
  x += dpp_d<0x4E>(x);      // quad_perm [2, 3, 0, 1]
  return x;
}

struct Quad16 {
  double a[4][16];          // slot s: row 4 s + j, columns 0 .. 4 s + 3 (past the row: unused)
  double hb[4], y[4], dinv[4], lbt[4], x[4];
  double hbb, y16;
};

// column J entries H[c][J], c = C .. 15, from lane c % 4 (slot c / 4), before step J scales them
template <int J, int C>
__device__ __forceinline__ void quad_col(const Quad16& Z, double (&hc)[16]) {
  if constexpr (C < 16) {
    hc[C] = quad_bcast<C % 4>(Z.a[C / 4][J]);
    quad_col<J, C + 1>(Z, hc);
  }
}

template <int J, int S>
__device__ __forceinline__ void quad_rows(Quad16& Z, const double (&hc)[16], double ij, double lb, double yj, int j) {
  if constexpr (S < 4) {
    // slot S holds row r = 4 S + j: below the pivot for S > J / 4, for S == J / 4 iff j > J % 4
    const bool below = S > J / 4 || (S == J / 4 && j > J % 4);
    const double l = below ? Z.a[S][J] * ij : 0.0;          // L[r][J]
#pragma unroll
    for (int c = J + 1; c < 4 * S + 4; ++c) Z.a[S][c] = fma(-l, hc[c], Z.a[S][c]);
    Z.hb[S] = below ? fma(-lb, Z.a[S][J], Z.hb[S]) : Z.hb[S];   // H[16][r] -= L[16][J] H[r][J]
    Z.y[S] = fma(-l, yj, Z.y[S]);
    if (below) Z.a[S][J] = l;
    quad_rows<J, S + 1>(Z, hc, ij, lb, yj, j);
  }
}

template <int J>
__device__ __forceinline__ void quad_steps(Quad16& Z, int j) {
  if constexpr (J < 16) {
    constexpr int SJ = J / 4, JJ = J % 4;
    const double dj = quad_bcast<JJ>(Z.a[SJ][J]);
    double ij = __builtin_amdgcn_rcp(dj);
    ij = fma(ij, fma(-dj, ij, 1.0), ij);
    ij = fma(ij, fma(-dj, ij, 1.0), ij);
    const double yj = quad_bcast<JJ>(Z.y[SJ]), hj = quad_bcast<JJ>(Z.hb[SJ]);
    const double lb = hj * ij;                              // L[16][J]
    double hc[16];
    quad_col<J, J + 1>(Z, hc);
    quad_rows<J, SJ>(Z, hc, ij, lb, yj, j);
    Z.hbb = fma(-lb, hj, Z.hbb);
    Z.y16 = fma(-lb, yj, Z.y16);
    if (j == JJ) {
      Z.dinv[SJ] = ij;
      Z.lbt[SJ] = lb;
    }
    quad_steps<J + 1>(Z, j);
  }
}

// L^T x = z from row 15 down: x_r = z_r - sum_{c > r} L[c][r] x_c - L[16][r] x_16
template <int R>
__device__ __forceinline__ void quad_back(Quad16& Z, const double (&z)[4], double x16, int j) {
  if constexpr (R >= 0) {
    constexpr int SR = R / 4, JR = R % 4;
    double p = 0.0;
#pragma unroll
    for (int s = SR; s < 4; ++s) {
      const bool below = s > SR || j > JR;                 // row 4 s + j > R
      p = below ? fma(Z.a[s][R], Z.x[s], p) : p;
    }
    p = quad_sum(p);
    if (j == JR) Z.x[SR] = z[SR] - p - Z.lbt[SR] * x16;
    quad_back<R - 1>(Z, z, x16, j);
  }
}

template <class M>
__global__ __launch_bounds__(64) void k_solve_quad(QueryArgs A, int64_t Q, double* __restrict__ rec,
                                                   double* __restrict__ x_out, int32_t* __restrict__ coupled) {
  static_assert(!M::ncf && M::K == 16, "MF k = 16");
  constexpr int K = M::K, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  const int lane = threadIdx.x, qd = lane >> 2, j = lane & 3, h = qd >> 1, sd = qd & 1;
  const int64_t q = (int64_t)blockIdx.x * 8 + h;
  const bool active = q < Q;
  const int64_t qc = active ? q : Q - 1;
  int32_t u = A.qu[qc], i = A.qi[qc];
  const bool okid = u >= 0 && u < A.U && i >= 0 && i < A.I;
  if (!okid) u = i = 0;
  const int32_t ent = sd ? i : u, oth = sd ? u : i;
  // the block's loads first (rows 4 s + j of the packed triangle, their bias-row entries, the
  // bias diagonal, the rhs), then the list lengths and the pair probe
  const double* __restrict__ G = A.gram[sd] + (int64_t)ent * GSP;
  const float* __restrict__ Eo = A.t[sd ? 0 : 1] + (int64_t)oth * K;
  Quad16 Z;
  double vv[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int r = 4 * s + j;
    const double* __restrict__ Gr = G + (r * (r + 1)) / 2;
#pragma unroll
    for (int c = 0; c < 4 * s + 4; ++c) Z.a[s][c] = Gr[c <= r ? c : r];
    Z.hb[s] = G[tri(K, r)];
    vv[s] = (double)Eo[r];
  }
  Z.hbb = G[tri(K, K)];
  const int64_t n = okid ? (A.ptr[0][u + 1] - A.ptr[0][u]) + (A.ptr[1][i + 1] - A.ptr[1][i]) : 0;
  double cdup = 0.0, rsum = 0.0;
  if (n > 0) A.pairs.lookup((unsigned long long)u * (unsigned long long)A.I + (unsigned long long)i, cdup, rsum);
  // H block = (2/n) Gram + wd on the embedding coordinates + damping
  const double s2n = n > 0 ? 2.0 / (double)n : 0.0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    const int r = 4 * s + j;
#pragma unroll
    for (int c = 0; c < 4 * s + 4; ++c) Z.a[s][c] = c <= r ? fma(Z.a[s][c], s2n, c == r ? A.wd + A.damping : 0.0) : 0.0;
    Z.hb[s] *= s2n;
    Z.y[s] = vv[s];
    Z.dinv[s] = Z.lbt[s] = Z.x[s] = 0.0;
  }
  Z.hbb = fma(Z.hbb, s2n, A.damping);
  Z.y16 = 1.0;
  quad_steps<0>(Z, j);
  double i16 = __builtin_amdgcn_rcp(Z.hbb);
  i16 = fma(i16, fma(-Z.hbb, i16, 1.0), i16);
  i16 = fma(i16, fma(-Z.hbb, i16, 1.0), i16);
  const double x16 = Z.y16 * i16;
  double z[4];
#pragma unroll
  for (int s = 0; s < 4; ++s) z[s] = Z.y[s] * Z.dinv[s];
  quad_back<15>(Z, z, x16, j);
  // record pieces: theta block, x.v, wd x.theta, r-hat(u,i) (sums over the query's two systems:
  // the quad, then the neighbouring quad)
  const float* __restrict__ Es = A.t[sd] + (int64_t)ent * K;
  double th[4], cq = 0.0, xg = j == 0 ? x16 : 0.0, pv = 0.0;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    th[s] = (double)Es[4 * s + j];
    cq = fma(Z.x[s], th[s], cq);
    xg = fma(Z.x[s], vv[s], xg);
    pv = fma(th[s], vv[s], pv);
  }
  cq = quad_sum(cq);
  xg = quad_sum(xg);
  pv = quad_sum(pv);
  cq = (cq + __shfl_xor(cq, 4)) * A.wd;
  xg += __shfl_xor(xg, 4);
  const double bself = (double)A.t[2 + sd][ent];
  const double gb = (double)A.t[4][0];
  const double bpair = bself + __shfl_xor(bself, 4);
  if (!active) return;
  if (n == 0) {
    if (x_out) {
#pragma unroll
      for (int s = 0; s < 4; ++s) x_out[q * D + M::ref_index(sd * Ds + 4 * s + j)] = NAN;
      if (j == 0) x_out[q * D + M::ref_index(sd * Ds + K)] = NAN;
    }
    if (sd == 0 && j == 0) rec[q * M::R] = NAN;
    return;
  }
  if (cdup > 0.0) {               // the test pair is a train row: the full-D k_solve finishes it
    if (sd == 0 && j == 0) {
      const int slot = atomicAdd(coupled, 1);
      coupled[1 + slot] = (int32_t)q;
    }
    return;
  }
  double* __restrict__ R = rec + q * M::R;
  if (sd == 0 && j == 0) {
    R[0] = 1.0 / (double)n;
    R[1] = cq;
    R[2] = xg;
    R[3] = pv + bpair + gb;        // r-hat(u,i)
  }
  double* __restrict__ S = R + 4 + sd * M::SB;
#pragma unroll
  for (int s = 0; s < 4; ++s) {
    S[4 * s + j] = th[s];
    S[K + 4 * s + j] = Z.x[s];
  }
  if (j == 0) {
    S[2 * K] = bself + gb;
    S[2 * K + 1] = x16;
    S[2 * K + 2] = (double)oth;
  }
  if (x_out) {
#pragma unroll
    for (int s = 0; s < 4; ++s) x_out[q * D + M::ref_index(sd * Ds + 4 * s + j)] = Z.x[s];
    if (j == 0) x_out[q * D + M::ref_index(sd * Ds + K)] = x16;
  }
}

// ------------------------------------------------------------------------------------
// MF, k <= 16: thread-per-system solve.  Every lane owns one (query, side) block of
// H_t (user block for even lanes, item block for odd lanes) and factors it with
// LDL^T entirely in registers (153 doubles at k=16, fully unrolled), then solves.  A
// query whose test pair is a train row couples the blocks: it is appended to the
// `coupled` list and solved afterwards by k_solve (one wave, full D).
// ------------------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(64) void k_solve_tps(QueryArgs A, int64_t Q, double* __restrict__ rec,
                                                  double* __restrict__ x_out, int32_t* __restrict__ coupled) {
  static_assert(!M::ncf, "thread-per-system solve is the MF path");
  constexpr int K = M::K, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  const int lane = threadIdx.x;
  const int64_t sys = (int64_t)blockIdx.x * 64 + lane;
  const int64_t q = sys >> 1;
  const int side = (int)(sys & 1);
  const bool active = q < Q;
  int32_t u = 0, i = 0;
  int64_t n = 0;
  if (active) {
    u = A.qu[q];
    i = A.qi[q];
    if (u >= 0 && u < A.U && i >= 0 && i < A.I)
      n = (A.ptr[0][u + 1] - A.ptr[0][u]) + (A.ptr[1][i + 1] - A.ptr[1][i]);
    else
      u = i = 0;
  }
  const int32_t ent = side == 0 ? u : i;       // this block's entity
  const int32_t oth = side == 0 ? i : u;       // the other endpoint of the test pair
  const float* Eself = side == 0 ? A.t[0] : A.t[1];
  const float* Eoth = side == 0 ? A.t[1] : A.t[0];
  const float* Bself = side == 0 ? A.t[2] : A.t[3];
  // the cached block's loads go out first: they overlap the pair lookup's probe chain
  const double* G = A.gram[side] + (int64_t)ent * GSP;
  double h[GS];
#define HS(t) h[(t)]
#pragma unroll
  for (int t = 0; t < GS; ++t) HS(t) = G[t];
  double cdup = 0.0, rsum = 0.0;
  if (active && n > 0)
    A.pairs.lookup((unsigned long long)u * (unsigned long long)A.I + (unsigned long long)i, cdup, rsum);
  if (active && n > 0 && cdup > 0.0 && side == 0) {
    const int slot = atomicAdd(coupled, 1);
    coupled[1 + slot] = (int32_t)q;
  }
  if (active && n == 0) {
    if (x_out)
      for (int a = 0; a < Ds; ++a) x_out[q * D + M::ref_index(side * Ds + a)] = NAN;
    if (side == 0) rec[q * M::R] = NAN;
  }
  const bool work = active && n > 0 && cdup == 0.0;

  // H block = (2/n) Gram + wd on the embedding coordinates + damping, in registers (fully
  // unrolled, every index constant)
  const double s2n = n > 0 ? 2.0 / (double)n : 0.0;
#pragma unroll
  for (int t = 0; t < GS; ++t) HS(t) *= s2n;
#pragma unroll
  for (int r = 0; r < Ds; ++r) HS(tri(r, r)) += (r < K ? A.wd : 0.0) + A.damping;

  // right-looking LDL^T: column j holds L[., j], the diagonal holds d
#pragma unroll
  // (the diagonal keeps 1/d: v_rcp_f64 + two Newton steps instead of an IEEE division
  // sequence on the critical path, and the forward solve multiplies by it)
  for (int j = 0; j < Ds; ++j) {
    const double dj = HS(tri(j, j));
    double inv = __builtin_amdgcn_rcp(dj);
    inv = fma(inv, fma(-dj, inv, 1.0), inv);
    inv = fma(inv, fma(-dj, inv, 1.0), inv);
#pragma unroll
    for (int r = j + 1; r < Ds; ++r) {
      const double lr = HS(tri(r, j)) * inv;
#pragma unroll
      for (int c = j + 1; c <= r; ++c) HS(tri(r, c)) = fma(-lr, HS(tri(c, j)), HS(tri(r, c)));
    }
#pragma unroll
    for (int r = j + 1; r < Ds; ++r) HS(tri(r, j)) *= inv;
    HS(tri(j, j)) = inv;
  }
  // v block: user side [q_i ; 1], item side [p_u ; 1]  (gnn:155, mf:194)
  double x[Ds];
  load_row_f32<K>(Eoth + (int64_t)oth * K, x);
  x[K] = 1.0;
#pragma unroll
  for (int j = 0; j < Ds; ++j)
#pragma unroll
    for (int r = j + 1; r < Ds; ++r) x[r] = fma(-HS(tri(r, j)), x[j], x[r]);
#pragma unroll
  for (int j = 0; j < Ds; ++j) x[j] *= HS(tri(j, j));
#pragma unroll
  for (int j = Ds - 1; j >= 0; --j)
#pragma unroll
    for (int c = 0; c < j; ++c) x[c] = fma(-HS(tri(j, c)), x[j], x[c]);
#undef HS

  // record pieces: theta block, x.v, wd x.theta, r-hat(u,i)
  double th[K], vv[K];
  load_row_f32<K>(Eself + (int64_t)ent * K, th);
  load_row_f32<K>(Eoth + (int64_t)oth * K, vv);
  const double bself = (double)Bself[ent];
  const double gb = (double)A.t[4][0];
  double cq = 0.0, xg = x[K], pv = 0.0;
#pragma unroll
  for (int a = 0; a < K; ++a) {
    cq = fma(x[a], th[a], cq);
    xg = fma(x[a], vv[a], xg);
    pv = fma(th[a], vv[a], pv);
  }
  cq *= A.wd;
  cq += __shfl_xor(cq, 1);
  xg += __shfl_xor(xg, 1);
  const double bpair = bself + __shfl_xor(bself, 1);
  if (!work) return;
  double* R = rec + q * M::R;
  if (side == 0) {
    R[0] = 1.0 / (double)n;
    R[1] = cq;
    R[2] = xg;
    R[3] = pv + bpair + gb;        // r-hat(u,i)
  }
  double* S = R + 4 + side * M::SB;
#pragma unroll
  for (int a = 0; a < K; ++a) {
    S[a] = th[a];
    S[K + a] = x[a];
  }
  S[2 * K] = bself + gb;
  S[2 * K + 1] = x[K];
  S[2 * K + 2] = (double)oth;
  if (x_out)
#pragma unroll
    for (int a = 0; a < Ds; ++a) x_out[q * D + M::ref_index(side * Ds + a)] = x[a];
}


// ------------------------------------------------------------------------------------
// MF Gram on the f64 matrix cores: one wave per entity, 4 list rows per
// v_mfma_f64_16x16x4_f64.  Lane l holds G[t0 + l/16][16 c + l%16] of the gathered
// other-side embeddings, which is both the A (= G^T) and the B operand of
// C += G^T G; the bias row (sums) and count come from VALU adds.
// C/D map (f64 16x16x4): col = l & 15, row = (l >> 4) + 4 r.
// ------------------------------------------------------------------------------------
// both sides' Gram work in one launch: blocks [0, n_items[0]) users, the rest items
struct GramSides {
  int64_t n_items[2];
  const int32_t* items[2];
  const int64_t* ptr[2];
  const int32_t* other[2];
  const float* emb_other[2];
  double* gram[2];
  double* part[2];
  // NCF (k_ncf_gram_rows): stored g_mlp rows per side, W3, list length N
  const double* lgm[2];
  const float* W3;
  int64_t N;
  // fia_prepare_for (small k): only the entities marked here (users [0, U), items [U, U+I))
  // get their Gram caches / per-position rows; nullptr = every entity
  const uint8_t* mark;
  int64_t moff[2];
  __device__ bool skip(int sd, int32_t e) const { return mark && !mark[moff[sd] + e]; }
  // MF k in {32, 64} (k_gram_mf_mfma): the residual e_p = r-hat_p - y_p of every list
  // position of a cached entity into lres[sd * N + p] for k_score_mf_mfma (nullptr: none)
  const float* emb_self[2];
  const float* rating[2];
  const float* bias[2];       // user, item bias tables
  const float* gb;
  double* lres;
};


template <class M>
__global__ __launch_bounds__(64) __attribute__((amdgpu_waves_per_eu(2))) void k_gram_mf_mfma(GramSides GSd) {
  constexpr int K = M::K, Ds = M::Ds, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  constexpr int NT = (K + 15) / 16;               // 16-wide column tiles
  constexpr int NP = NT * (NT + 1) / 2;           // upper tile pairs
  // MFMA row-quads gathered ahead per batch (k = 64: 6, so the double-buffered rows, the
  // residual pass and the 10 accumulator tiles fit two waves per SIMD)
  constexpr int SUB = NT <= 2 ? 16 : NT == 3 ? 8 : 6;
  const int sd = (int64_t)blockIdx.x >= GSd.n_items[0] ? 1 : 0;
  const int64_t w = (int64_t)blockIdx.x - (sd ? GSd.n_items[0] : 0);
  if (w >= GSd.n_items[sd]) return;
  const int32_t* __restrict__ items = GSd.items[sd];
  const int64_t* __restrict__ ptr = GSd.ptr[sd];
  const int32_t* __restrict__ other = GSd.other[sd];
  const float* __restrict__ emb_other = GSd.emb_other[sd];
  double* __restrict__ gram = GSd.gram[sd];
  double* __restrict__ part = GSd.part[sd];
  const int32_t e = items[4 * w], start = items[4 * w + 1], len = items[4 * w + 2], slot = items[4 * w + 3];
  if (GSd.skip(sd, e)) return;
  const int lane = threadIdx.x;
  const int col = lane & 15, grp = lane >> 4;
  const int32_t* ids = other + ptr[e] + start;
  d4_t acc[NP];
#pragma unroll
  for (int p = 0; p < NP; ++p) acc[p] = d4_t{0.0, 0.0, 0.0, 0.0};
  double sum[NT];
#pragma unroll
  for (int t = 0; t < NT; ++t) sum[t] = 0.0;
  // one coalesced load of 4*SUB row ids per batch, every row-quad's gather in flight at
  // once.  k >= 32: software-pipelined (ids two batches ahead, gathers one batch ahead;
  // 20M MF k=64 prepare 8.0 -> 6.7 ms); k <= 16 lists are mostly one or two batches and
  // the look-ahead costs more than it hides (ml-1m-ex 57 -> 65 us)
  auto ids_at = [&](int t0) -> int32_t { return (lane < 4 * SUB && t0 + lane < len) ? ids[t0 + lane] : -1; };
  auto gather = [&](int32_t id, double (&val)[SUB][NT]) {
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      const int32_t o = __shfl(id, 4 * sb + grp);
      const float* src = emb_other + (int64_t)(o < 0 ? 0 : o) * K;
#pragma unroll
      for (int t = 0; t < NT; ++t) val[sb][t] = (o >= 0 && 16 * t + col < K) ? (double)src[16 * t + col] : 0.0;
    }
  };
  auto accumulate = [&](const double (&val)[SUB][NT]) {
#pragma unroll
    for (int sb = 0; sb < SUB; ++sb) {
      int p = 0;
#pragma unroll
      for (int ta = 0; ta < NT; ++ta) {
        sum[ta] += val[sb][ta];
#pragma unroll
        for (int tb = ta; tb < NT; ++tb, ++p)
          acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(val[sb][ta], val[sb][tb], acc[p], 0, 0, 0);
      }
    }
  };
  if constexpr (K >= 32) {
    // the residual of each gathered row (mf:89-116): the entity's own row dotted with it --
    // lane (grp, col) holds coordinates 16 t + col of row 4 sb + grp, so a row's dot is a
    // 16-lane DPP sum; lane l < 4 SUB then owns batch row l (its list entry, rating and the
    // other side's bias, loaded with the row's gather one batch ahead).  The products and the
    // sum order are the same from either side's list, so both copies have the same bits.
    const bool want_res = GSd.lres != nullptr;
    const float* __restrict__ es = GSd.emb_self[sd] + (int64_t)e * K;
    double eself[NT];
#pragma unroll
    for (int t = 0; t < NT; ++t) eself[t] = 16 * t + col < K ? (double)es[16 * t + col] : 0.0;
    const double bself = want_res ? (double)GSd.bias[sd][e] : 0.0, gbias = want_res ? (double)GSd.gb[0] : 0.0;
    const float* __restrict__ bother = GSd.bias[1 - sd];
    const int64_t lp0 = ptr[e] + start;
    const float* __restrict__ ratp = GSd.rating[sd] + lp0;
    auto row_loads = [&](int32_t id, int t0, float& y, float& bo) {
      const bool ok = want_res && lane < 4 * SUB && t0 + lane < len;
      y = ok ? ratp[t0 + lane] : 0.0f;
      bo = ok && id >= 0 ? bother[id] : 0.0f;
    };
    auto residuals = [&](const double (&val)[SUB][NT], float y, float bo, int t0) {
      double r = 0.0;
#pragma unroll
      for (int sb = 0; sb < SUB; ++sb) {
        double part = 0.0;
#pragma unroll
        for (int t = 0; t < NT; ++t) part = fma(eself[t], val[sb][t], part);
        const double v = __shfl(row_sum16(part), 16 * (lane & 3));
        r = (lane >> 2) == sb ? v : r;
      }
      if (lane < 4 * SUB && t0 + lane < len) {
        const double bu = sd == 0 ? bself : (double)bo, bi = sd == 0 ? (double)bo : bself;
        GSd.lres[sd * GSd.N + lp0 + t0 + lane] = ((r + bu) + bi) + gbias - (double)y;
      }
    };
    double val[SUB][NT];
    int32_t id_c = ids_at(0);
    gather(id_c, val);
    float y_c, bo_c;
    row_loads(id_c, 0, y_c, bo_c);
    int32_t id_n = ids_at(4 * SUB);
    for (int t0 = 0; t0 < len; t0 += 4 * SUB) {
      const int32_t id_nn = ids_at(t0 + 8 * SUB);
      double vn[SUB][NT];
      gather(id_n, vn);                          // next batch (ids -1 past the end)
      float y_n, bo_n;
      row_loads(id_n, t0 + 4 * SUB, y_n, bo_n);
      if (want_res) residuals(val, y_c, bo_c, t0);
      accumulate(val);
#pragma unroll
      for (int sb = 0; sb < SUB; ++sb)
#pragma unroll
        for (int t = 0; t < NT; ++t) val[sb][t] = vn[sb][t];
      y_c = y_n;
      bo_c = bo_n;
      id_n = id_nn;
    }
  } else {
    // k <= 16 (a work item is <= 256 rows = 4 batches): every batch's row ids loaded up front
    // (one latency instead of one per batch), the gathers batch by batch
    constexpr int NB = 4;
    int32_t idb[NB];
#pragma unroll
    for (int b = 0; b < NB; ++b) idb[b] = ids_at(4 * SUB * b);
#pragma unroll
    for (int b = 0; b < NB; ++b) {
      if (4 * SUB * b >= len) break;
      double val[SUB][NT];
      gather(idb[b], val);
      accumulate(val);
    }
    for (int t0 = 4 * SUB * NB; t0 < len; t0 += 4 * SUB) {      // (longer work items)
      double val[SUB][NT];
      gather(ids_at(t0), val);
      accumulate(val);
    }
  }
  double* out = slot < 0 ? gram + (int64_t)e * GSP : part + (int64_t)slot * GSP;
  int p = 0;
#pragma unroll
  for (int ta = 0; ta < NT; ++ta) {
#pragma unroll
    for (int tb = ta; tb < NT; ++tb, ++p) {
#pragma unroll
      for (int rr = 0; rr < 4; ++rr) {
        const int ci = 16 * ta + grp + 4 * rr;    // C row -> Gram column index (tile ta)
        const int rj = 16 * tb + col;             // C col -> Gram row index (tile tb)
        if (ci < K && rj < K && rj >= ci) out[tri(rj, ci)] = acc[p][rr];
      }
    }
  }
  // bias row: Gram[K][c] = sum over rows of G[.][c]; Gram[K][K] = row count
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    double s = sum[t];
    s += __shfl_xor(s, 16);
    s += __shfl_xor(s, 32);
    if (grp == 0 && 16 * t + col < K) out[tri(K, 16 * t + col)] = s;
  }
  if (lane == 0) out[tri(K, K)] = (double)len;
}

// ------------------------------------------------------------------------------------
// NCF per list position + entity Gram, one pass (ncf:102-145, TF ReluGrad masks).  A wave
// takes one work item (<= gchunk positions of one entity's list, both sides in one
// launch) in slabs of 16 positions p, e = the entity, o = other(p):
//   z1 = (L1_self[e] + b1) + L1_other[o],  z2 = relu(z1) W2 + b2,  d2 = 1[z2 > 0] W3m,
//   d1 = 1[z1 > 0] (W2 d2),  g_mlp = W1_side d1,  e_p = W3m.relu(z2) + W3g.(Gs_e*Go_o) + b3 - y,
//   Gram_e += g g^T over g = [g_mlp ; W3g * Go_o]
// and stores g_mlp to lgm[a * N + p] (coordinate-major) and e_p to lres[p] for scoring.
// All products run on v_mfma_f64_16x16x4_f64.  The MLP runs transposed -- out^T = W . in^T
// with the 16 positions along n -- so the weights are per-lane A operands loaded once
// per wave and each product's C registers are the next product's B operand as they stand
// (C register r = rows (l>>4) + 4r = the next k-slice r).  The last product runs the
// other way round, g_mlp = d1 . W1_side^T (the same per-lane W1 values as B operand), so
// its C register r holds positions 4r + (l>>4) x coordinates l&15 -- exactly the Gram
// MFMA's operand for row-quad r.  No LDS, no transposes.
// Map: lane l supplies A[l&15][l>>4] and B[l>>4][l&15]; C register r = out[(l>>4)+4r][l&15].
// ------------------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(64) void k_ncf_gram_rows(GramSides GSd, const float* __restrict__ W1,
                                                      const float* __restrict__ b1, const float* __restrict__ W2,
                                                      const float* __restrict__ b2, const float* __restrict__ b3,
                                                      const double* __restrict__ l1u, const double* __restrict__ l1i,
                                                      const float* __restrict__ rat0, const float* __restrict__ rat1,
                                                      double* __restrict__ lres) {
  constexpr int K = M::K, H = K / 2, KK = K / 4, HK = (H + 3) / 4, KT = (K + 15) / 16;
  constexpr int Ds = M::Ds, GS = Ds * (Ds + 1) / 2, GSP = (GS + 1) & ~1;
  constexpr int NT = Ds / 16, NP = NT * (NT + 1) / 2;
  static_assert(M::ncf && K % 8 == 0 && H <= 16 && Ds % 16 == 0, "NCF k in {8, 16, 32}");
  const float* __restrict__ W3 = GSd.W3;
  const int64_t N = GSd.N;
  const int lane = threadIdx.x, m = lane & 15, kq = lane >> 4;
  const int64_t n_all = GSd.n_items[0] + GSd.n_items[1];
  // side-independent weight operands (per lane, once per wave)
  double aW2t[KK], aW2[KT][HK], cb2[4], cw3[4], w3gk[KK], b1v[KK], w3gt[NT];
#pragma unroll
  for (int kk = 0; kk < KK; ++kk) {
    const int c = kq + 4 * kk;
    aW2t[kk] = m < H ? (double)W2[c * H + m] : 0.0;           // A[h][c] = W2[c][h]
    w3gk[kk] = (double)W3[H + c];
    b1v[kk] = (double)b1[c];
  }
#pragma unroll
  for (int t = 0; t < KT; ++t) {
    const int row = m + 16 * t;
#pragma unroll
    for (int kk = 0; kk < HK; ++kk) {
      const int h = kq + 4 * kk;
      aW2[t][kk] = row < K && h < H ? (double)W2[row * H + h] : 0.0;          // A[c][h] = W2[c][h]
    }
  }
#pragma unroll
  for (int r = 0; r < 4; ++r) {
    const int h = kq + 4 * r;
    cb2[r] = h < H ? (double)b2[h] : 0.0;
    cw3[r] = h < H ? (double)W3[h] : 0.0;
  }
#pragma unroll
  for (int t = 0; t < NT; ++t) {
    const int co = 16 * t + m;
    w3gt[t] = co >= K ? (double)W3[H + co - K] : 0.0;
  }
  const double bias3 = (double)b3[0];
  int cur_side = -1;
  double aW1[KT][KK];          // W1_side[a = m + 16t][c = kq + 4kk]: A of nothing, B of g_mlp = d1 W1^T
  for (int64_t w = blockIdx.x; w < n_all; w += gridDim.x) {
    const int sd = w >= GSd.n_items[0] ? 1 : 0;
    const int64_t wi = w - (sd ? GSd.n_items[0] : 0);
    if (sd != cur_side) {
      cur_side = sd;
#pragma unroll
      for (int t = 0; t < KT; ++t)
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) {
          const int a = m + 16 * t;
          aW1[t][kk] = a < K ? (double)W1[(int64_t)(sd * K + a) * K + kq + 4 * kk] : 0.0;
        }
    }
    const int32_t* __restrict__ it = GSd.items[sd] + 4 * wi;
    const int32_t e = it[0], start = it[1], len = it[2], slot = it[3];
    if (GSd.skip(sd, e)) continue;
    const int64_t lb = GSd.ptr[sd][e] + start;
    const int32_t* __restrict__ ids = GSd.other[sd] + lb;
    const float* __restrict__ rat = (sd ? rat1 : rat0) + lb;
    const float* __restrict__ Go = GSd.emb_other[sd];
    const float* __restrict__ Gs = GSd.emb_other[1 - sd] + (int64_t)e * K;     // own gmf row
    const double* __restrict__ Ls = (sd ? l1i : l1u) + (int64_t)e * K;
    const double* __restrict__ L1o = sd ? l1u : l1i;
    double* __restrict__ lgp = const_cast<double*>(GSd.lgm[sd]) + lb;
    int32_t* __restrict__ lmk = reinterpret_cast<int32_t*>(const_cast<double*>(GSd.lgm[sd])) + lb;   // mask path
    double* __restrict__ lrp = lres + (int64_t)sd * N + lb;
    double zs[KK], gsk[KK];     // own-entity terms for this lane's coordinates
#pragma unroll
    for (int kk = 0; kk < KK; ++kk) {
      zs[kk] = Ls[kq + 4 * kk] + b1v[kk];
      gsk[kk] = w3gk[kk] * (double)Gs[kq + 4 * kk];
    }
    d4_t acc[NP];
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p] = d4_t{0.0, 0.0, 0.0, 0.0};
    // Software pipeline over the slabs: the list ids run two slabs ahead and the gathers
    // one slab ahead (they only depend on the ids), so a slab waits on no memory round trip.
    // Per slab and lane: lo = L1_other[o_m][kq + 4kk], gf = Go[o_m][kq + 4kk] (residual),
    // gg[r][t] = Go[o_(4r+kq)][16t + m - k] (Gram operand of the gmf coordinates).
    const int lastp = len - 1;
    int32_t o = ids[m < lastp ? m : lastp];
    int32_t o_n = ids[16 + m < lastp ? 16 + m : lastp];
    double lo[KK];
    float gf[KK], gg[4][NT];
    auto gather = [&](int32_t oo, double (&lo_)[KK], float (&gf_)[KK], float (&gg_)[4][NT]) {
      const double* __restrict__ Lo = L1o + (int64_t)oo * K;
      const float* __restrict__ Gom = Go + (int64_t)oo * K;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        lo_[kk] = Lo[kq + 4 * kk];
        gf_[kk] = Gom[kq + 4 * kk];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int32_t orow = __shfl(oo, 4 * r + kq);
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int co = 16 * t + m;
          gg_[r][t] = 0.f;
          if (16 * t + 15 >= K && co >= K) gg_[r][t] = Go[(int64_t)orow * K + co - K];
        }
      }
    };
    gather(o, lo, gf, gg);
    for (int s0 = 0; s0 < len; s0 += 16) {
      const bool ok = s0 + m < len;
      const int32_t o_nn = ids[s0 + 32 + m < lastp ? s0 + 32 + m : lastp];
      double lo_n[KK];
      float gf_n[KK], gg_n[4][NT];
      gather(o_n, lo_n, gf_n, gg_n);       // next slab (a harmless repeat past the end)
      double z1[KK];
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) z1[kk] = ok ? zs[kk] + lo[kk] : 0.0;
      d4_t z2 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
      for (int kk = 0; kk < KK; ++kk)
        z2 = __builtin_amdgcn_mfma_f64_16x16x4f64(aW2t[kk], z1[kk] > 0.0 ? z1[kk] : 0.0, z2, 0, 0, 0);
      double mlp = 0.0, d2[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const double z = z2[r] + cb2[r];
        const bool on = z > 0.0;
        mlp = fma(cw3[r], on ? z : 0.0, mlp);
        d2[r] = on ? cw3[r] : 0.0;
      }
      double d1[KK];
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        d4_t t1 = {0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < HK; ++kk) t1 = __builtin_amdgcn_mfma_f64_16x16x4f64(aW2[t][kk], d2[kk], t1, 0, 0, 0);
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (4 * t + r < KK) d1[4 * t + r] = z1[4 * t + r] > 0.0 ? t1[r] : 0.0;
      }
      // g_mlp = d1 W1_side^T: C register r = positions 4r + kq, coordinates m + 16t
      d4_t gm[KT];
#pragma unroll
      for (int t = 0; t < KT; ++t) {
        gm[t] = d4_t{0.0, 0.0, 0.0, 0.0};
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) gm[t] = __builtin_amdgcn_mfma_f64_16x16x4f64(d1[kk], aW1[t][kk], gm[t], 0, 0, 0);
      }
      if constexpr (mask_path<M>()) {
        // ReLU masks of position m: lane (m, kq) holds z1 at c = kq + 4kk and z2 at h = kq + 4r
        int mk = 0;
#pragma unroll
        for (int kk = 0; kk < KK; ++kk) mk |= z1[kk] > 0.0 ? 1 << (kq + 4 * kk) : 0;
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (kq + 4 * r < H) mk |= z2[r] + cb2[r] > 0.0 ? 1 << (K + kq + 4 * r) : 0;   // d2's `on`
        mk |= __shfl_xor(mk, 16);
        mk |= __shfl_xor(mk, 32);
        if (kq == 0 && ok) lmk[s0 + m] = mk;
      }
      // residual of position m (mlp and the gmf dot are split over the 4 lane groups)
      double gmf = 0.0;
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) gmf = fma(gsk[kk], (double)gf[kk], gmf);
      double re = mlp + gmf;
      re += __shfl_xor(re, 16);
      re += __shfl_xor(re, 32);
      if (kq == 0 && ok) lrp[s0 + m] = re + bias3 - (double)rat[s0 + m];
      // Gram row-quads r: positions 4r + kq
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const int pr = s0 + 4 * r + kq;
        const bool okr = pr < len;
        double val[NT];
#pragma unroll
        for (int t = 0; t < NT; ++t) {
          const int co = 16 * t + m;
          const double gv = gm[t < KT ? t : KT - 1][r];
          double x;
          if (co < K) {
            x = gv;
            if constexpr (!mask_path<M>())
              if (okr) lgp[(int64_t)co * N + pr] = gv;
          } else {
            x = w3gt[t] * (double)gg[r][t];
          }
          val[t] = okr ? x : 0.0;
        }
        int p = 0;
#pragma unroll
        for (int ta = 0; ta < NT; ++ta)
#pragma unroll
          for (int tb = ta; tb < NT; ++tb, ++p)
            acc[p] = __builtin_amdgcn_mfma_f64_16x16x4f64(val[ta], val[tb], acc[p], 0, 0, 0);
      }
#pragma unroll
      for (int kk = 0; kk < KK; ++kk) {
        lo[kk] = lo_n[kk];
        gf[kk] = gf_n[kk];
      }
#pragma unroll
      for (int r = 0; r < 4; ++r)
#pragma unroll
        for (int t = 0; t < NT; ++t) gg[r][t] = gg_n[r][t];
      o_n = o_nn;
    }
    double* out = slot < 0 ? GSd.gram[sd] + (int64_t)e * GSP : GSd.part[sd] + (int64_t)slot * GSP;
    int p = 0;
#pragma unroll
    for (int ta = 0; ta < NT; ++ta)
#pragma unroll
      for (int tb = ta; tb < NT; ++tb, ++p)
#pragma unroll
        for (int rr = 0; rr < 4; ++rr) {
          const int ci = 16 * ta + kq + 4 * rr;    // C row -> Gram column index (tile ta)
          const int rj = 16 * tb + m;              // C col -> Gram row index (tile tb)
          if (rj >= ci) out[gidx<M>(rj, ci)] = acc[p][rr];
        }
  }
}

// Sum the partial Grams of split lists in slot order (deterministic); both sides in one
// launch (blocks [0, n_comb0) the user side).
__global__ __launch_bounds__(256) void k_gram_combine(int64_t n_comb0, const int32_t* __restrict__ comb0,
                                                     const double* __restrict__ part0, double* __restrict__ gram0,
                                                     int64_t n_comb1, const int32_t* __restrict__ comb1,
                                                     const double* __restrict__ part1, double* __restrict__ gram1,
                                                     int GS, int GSP, const uint8_t* __restrict__ mark, int64_t moff1) {
  const int sd = (int64_t)blockIdx.x >= n_comb0 ? 1 : 0;
  const int64_t w = (int64_t)blockIdx.x - (sd ? n_comb0 : 0);
  if (w >= (sd ? n_comb1 : n_comb0)) return;
  const int32_t* __restrict__ comb = sd ? comb1 : comb0;
  const double* __restrict__ part = sd ? part1 : part0;
  double* __restrict__ gram = sd ? gram1 : gram0;
  const int32_t e = comb[4 * w], first = comb[4 * w + 1], ns = comb[4 * w + 2];
  if (mark && !mark[(sd ? moff1 : 0) + e]) return;
  // partials summed in slot order (deterministic), their loads issued 8 slots at a time
  // rather than one dependent round trip per slot; the last group's missing slots load slot
  // `first` and are weighted 0 (branch-free: a partial group is not a chain of round trips)
  for (int t = threadIdx.x; t < GS; t += blockDim.x) {
    const double* __restrict__ pt = part + (int64_t)first * GSP + t;
    double s = 0.0;
    for (int k = 0; k < ns; k += 8) {
      double v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) v[j] = pt[(int64_t)(k + j < ns ? k + j : 0) * GSP];
#pragma unroll
      for (int j = 0; j < 8; ++j) s += k + j < ns ? v[j] : 0.0;
    }
    gram[(int64_t)e * GSP + t] = s;
  }
}

// ------------------------------------------------------------------------------------
// Scoring (the dominant, HBM-streaming kernel).  Per related rating j of a query:
//   influence_j = (2 e_j s_j + c_q) / n,  s_j = x . g_j,  e_j = r-hat_j - y_j
// (mf:240-246: x . grad L_j / n with grad L_j = 2 e_j g_j + wd * M * theta_t); the K best
// of every chunk (|influence| desc, position asc) go to its candidate slots.
// ------------------------------------------------------------------------------------

// ------------------------------------------------------------------------------------
// Entity-shared scoring (MF k >= 32, NCF).  A work item is one chunk (<= kChunk ratings) of
// ONE entity's list (user list R_u or item list C_i) together with a block of the batch's
// queries that have that entity.  The list entries, the gathered other-side embedding rows
// and the per-rating residual e_j = r-hat_j - y_j depend on the train rating only, so they
// are loaded / computed once per work item and reused for every query in the block; per
// query only s_jq = x_q . g_j is new.  influence_jq = (2 e_j s_jq + c_q) / n_q
// (mf:240-246).  The test pair's own train row takes e and s from the query record
// (bit-identical copies, see k_solve).

// ------------------------------------------------------------------------------------
// MF k >= 32 entity-shared scoring with the query vectors read through the scalar cache.
// The work item (<= 256 ratings of one entity's list x <= 8 queries sharing the entity)
// needs, per query, x (k doubles) and a few header words -- the same for every lane.  In
// LDS every use is a broadcast read that still costs the LDS a full 64-lane transfer
// (with 4 rows per lane: one 16-B read per 8 FMAs, ~the LDS bandwidth of a CU); here they
// are s_load'ed into SGPRs and consumed as the SGPR operand of v_fma_f64, leaving LDS
// idle (20M MF k=64: 5.04 -> 4.74 ms per batch).  One candidate slot set per work item
// (spc = 1).
// ------------------------------------------------------------------------------------
// queries per entity-shared work item: 16 for MF k >= 64, where a work item's gathered
// rows (256 B each) are the dominant traffic and two query blocks would load them twice
template <class M>
constexpr int query_block() {
  return (!M::ncf && M::K >= 64) ? 16 : kQueryBlock;
}

template <class M>
__global__ __launch_bounds__(kScoreThreads) void k_score_grouped_mf(
    QueryArgs A, int64_t nE, const int64_t* __restrict__ wstart, const int32_t* __restrict__ witems,
    const int64_t* __restrict__ gstart, const int32_t* __restrict__ gq, const int64_t* __restrict__ qbase,
    const double* __restrict__ rec, int32_t* __restrict__ rel_idx, double* __restrict__ influence, int K_top,
    int32_t* __restrict__ cand_pos, double* __restrict__ cand_val) {
  static_assert(!M::ncf && M::K % 4 == 0, "MF, k a multiple of 4");
  constexpr int K = M::K, RT = kScoreRows, QB = query_block<M>(), CK = 4;
  constexpr int NSV = (K + 1 + 63) / 64;
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_items = wstart[nE];
  const int64_t stride = (int64_t)gridDim.x * (kScoreThreads / 64);
  for (int64_t wi = (int64_t)blockIdx.x * (kScoreThreads / 64) + wave; wi < n_items; wi += stride) {
    const int32_t g = witems[3 * wi], cidx = witems[3 * wi + 1], qblk = witems[3 * wi + 2];
    const int sd = g >= A.U ? 1 : 0;
    const int32_t e = sd ? (int32_t)(g - A.U) : g;
    const int64_t lb = A.ptr[sd][e] + (int64_t)cidx * kChunk;
    const int64_t rem = A.ptr[sd][e + 1] - lb;
    const int len = rem < kChunk ? (int)rem : kChunk;
    const int64_t gb = gstart[g] + (int64_t)qblk * QB;
    const int64_t gn = gstart[g + 1] - gb;
    const int nq = gn < QB ? (int)gn : QB;
    const int32_t* __restrict__ oth = A.other[sd] + lb;
    const float* __restrict__ rat = A.rating[sd] + lb;
    const int32_t* __restrict__ rw = A.row[sd] + lb;
    double selfv[NSV];
#pragma unroll
    for (int v = 0; v < NSV; ++v) {
      const int c = v * 64 + lane;
      const float* Es = sd == 0 ? A.t[0] : A.t[1];
      const float* Bs = sd == 0 ? A.t[2] : A.t[3];
      selfv[v] = c < K ? (double)Es[(int64_t)e * K + c] : (double)Bs[e];
    }
#define SV(c) readlane_d(selfv[(c) / 64], (c) % 64)
    int32_t o_[RT], row_[RT];
    float y_[RT], gb_[RT];
    bool ok_[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int idx = r * 64 + lane;
      ok_[r] = idx < len;
      const int li = ok_[r] ? idx : 0;
      o_[r] = oth[li];
      y_[r] = rat[li];
      row_[r] = rw[li];
    }
    const float* __restrict__ T = sd == 0 ? A.t[1] : A.t[0];
    const float* __restrict__ bt = sd == 0 ? A.t[3] : A.t[2];
#pragma unroll
    for (int r = 0; r < RT; ++r) gb_[r] = bt[o_[r]];
    // NQ = nq rounded up to a power of two: a static query count per path keeps the
    // accumulators in registers (padding columns repeat the last query, never written out)
    auto run = [&](auto nq_c) {
      constexpr int NQ = decltype(nq_c)::value;
      const double* __restrict__ xq[NQ];        // uniform: this side's x of each query
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const int32_t q = gq[gb + (j < nq ? j : nq - 1)];
        xq[j] = rec + (int64_t)q * M::R + 4 + sd * M::SB;
      }
      double ea[RT], acc[NQ][RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) {
        ea[r] = 0.0;
#pragma unroll
        for (int j = 0; j < NQ; ++j) acc[j][r] = 0.0;
      }
      float4 ga[RT];
#pragma unroll
      for (int r = 0; r < RT; ++r) ga[r] = *reinterpret_cast<const float4*>(T + (int64_t)o_[r] * K);
#pragma unroll 1
      for (int c0 = 0; c0 < K; c0 += CK) {
        float4 gn[RT];
        const int cn = c0 + CK < K ? c0 + CK : c0;
#pragma unroll
        for (int r = 0; r < RT; ++r) gn[r] = *reinterpret_cast<const float4*>(T + (int64_t)o_[r] * K + cn);
        double gd[RT][CK];
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          gd[r][0] = ga[r].x; gd[r][1] = ga[r].y; gd[r][2] = ga[r].z; gd[r][3] = ga[r].w;
        }
#pragma unroll
        for (int cc = 0; cc < CK; ++cc) {
          const double sc = SV(c0 + cc);
#pragma unroll
          for (int r = 0; r < RT; ++r) ea[r] = fma(sc, gd[r][cc], ea[r]);
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
#pragma unroll
          for (int cc = 0; cc < CK; ++cc) {
            const double xc = xq[j][K + c0 + cc];  // scalar load, SGPR operand
#pragma unroll
            for (int r = 0; r < RT; ++r) acc[j][r] = fma(xc, gd[r][cc], acc[j][r]);
          }
        }
#pragma unroll
        for (int r = 0; r < RT; ++r) ga[r] = gn[r];
      }
      {
        const double gbias = (double)A.t[4][0];
        const double bself = SV(K);
#pragma unroll
        for (int r = 0; r < RT; ++r) ea[r] = ea[r] + bself + (double)gb_[r] + gbias - (double)y_[r];
      }
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        if (j >= nq) continue;
        const int32_t q = gq[gb + j];
        const double* __restrict__ R = rec + (int64_t)q * M::R;
        const double inv_n = R[0], cq = R[1], xv = R[2], rhat_ui = R[3];
        const double xsb = xq[j][2 * K + 1], dup_o = xq[j][2 * K + 2];
        const int64_t* __restrict__ qb = qbase + 4 * (int64_t)q;
        const int64_t obj = qb[sd] + (int64_t)cidx * kChunk, cbj = qb[2 + sd] + cidx;
        const int64_t poj = sd ? qb[1] - qb[0] : 0;   // |R_u| precedes item-side positions
        double la[RT], lv[RT];
        int lp[RT];
#pragma unroll
        for (int r = 0; r < RT; ++r) {
          double ee = ea[r], ss = acc[j][r] + xsb;
          if ((double)o_[r] == dup_o) { ee = rhat_ui - (double)y_[r]; ss = xv; }
          const double infl = (2.0 * ee * ss + cq) * inv_n;
          const int idx = r * 64 + lane;
          if (ok_[r]) {
            if (influence) __builtin_nontemporal_store(infl, influence + obj + idx);
            if (rel_idx) __builtin_nontemporal_store(row_[r], rel_idx + obj + idx);
          }
          lp[r] = ok_[r] ? cidx * kChunk + idx : -1;
          la[r] = ok_[r] ? topk_key(infl) : -2.0;
          lv[r] = infl;
        }
        if (K_top > 0) {
          double pa = INFINITY;
          int pp = -1;
          for (int t = 0; t < K_top; ++t) {
            double ba = -2.0, bv = 0.0;
            int bp = 0x7fffffff;
#pragma unroll
            for (int r = 0; r < RT; ++r)
              if (lp[r] >= 0 && better(pa, pp, la[r], lp[r]) && better(la[r], lp[r], ba, bp)) {
                ba = la[r]; bp = lp[r]; bv = lv[r];
              }
            wave_best(ba, bp, bv);
            if (lane == 0) {
              const bool okk = ba > -1.5;
              const int64_t slot = cbj * K_top + t;
              cand_pos[slot] = okk ? (int32_t)(bp + poj) : -1;
              cand_val[slot] = okk ? bv : NAN;
            }
            pa = ba;
            pp = bp;
          }
        }
      }
    };
    if (nq <= 1) run(std::integral_constant<int, 1>{});
    else if (nq <= 2) run(std::integral_constant<int, 2>{});
    else if (nq <= 4) run(std::integral_constant<int, 4>{});
    else if (QB == 8 || nq <= 8) run(std::integral_constant<int, 8>{});
    else run(std::integral_constant<int, QB>{});
#undef SV
  }
}

// MF k in {32, 64}, K_top <= 1: k_score_mf_mfma (score_mfma.hip)

// NCF k <= 16 (mask path): T[m][c] = sum_e W2[c][e] W3m[e] [bit e of m], the d1 of a train
// row whose z2 ReLU mask is m (before its z1 mask), one thread per entry
template <class M>
__global__ __launch_bounds__(256) void k_ncf_d1_table(const float* __restrict__ W2, const float* __restrict__ W3,
                                                      double* __restrict__ tab) {
  constexpr int K = M::K, H = K / 2;
  const int t = blockIdx.x * 256 + threadIdx.x;
  if (t >= (1 << H) * K) return;
  const int m2 = t / K, c = t - m2 * K;
  double v = 0.0;
#pragma unroll
  for (int e = 0; e < H; ++e) v = fma((double)W2[c * H + e], (m2 >> e) & 1 ? (double)W3[e] : 0.0, v);
  tab[t] = v;
}

// NCF k <= 16 (mask path): the record's MLP block x_mlp -> y = W1_side^T x_mlp, one thread
// per (query, side), after every solve of the batch (k_score_ncf dots y with d1)
template <class M>
__global__ __launch_bounds__(256) void k_ncf_rec_y(int64_t Q, const float* __restrict__ W1, double* __restrict__ rec) {
  constexpr int K = M::K;
  // W1 as fp64 in LDS: read per use as a broadcast (the per-use scalar loads of the fp32
  // table exposed one memory latency per weight: 20 us at yelp-ex)
  __shared__ double w1[2 * K * K];
  for (int e = threadIdx.x; e < 2 * K * K; e += 256) w1[e] = (double)W1[e];
  __syncthreads();
  const int64_t t = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (t >= 2 * Q) return;
  const int64_t q = t >> 1;
  const int sd = (int)(t & 1);
  double* __restrict__ S = rec + q * M::R + 4 + sd * M::SB;
  double x[K];
#pragma unroll
  for (int a = 0; a < K; ++a) x[a] = S[a];
  const double* __restrict__ ws = w1 + sd * K * K;
#pragma unroll
  for (int c = 0; c < K; ++c) {
    double y = 0.0;
#pragma unroll
    for (int a = 0; a < K; ++a) y = fma(ws[a * K + c], x[a], y);
    S[c] = y;
  }
}

// ------------------------------------------------------------------------------------
// NCF entity-shared scoring.  Same work items, query blocks and outputs as
// k_score_grouped_mf, but nothing of the MLP is recomputed here: per list position the
// Gram pass stored e_j and, per list position, the ReLU masks (k <= 16; k = 32: g_mlp,j =
// W1_side . d1_j coordinate-major, every load a coalesced 512-B wave row), and the solve
// stored x_mlp (k <= 16: y = W1_side^T x_mlp after k_ncf_rec_y) and W3g * x_gmf, so
//   s_jq = y_q . d1_j + (W3g * x_gmf,q) . gmf_other(j)  =  x_mlp,q . g_mlp,j + ...   (ncf:193-280)
// with d1_j from the z1 mask and the table row of the z2 mask (k_ncf_d1_table, in LDS)
// is 2k FMAs per (rating, query) over the work item's 256 ratings (4 rows per lane).
// One candidate slot set per work item (spc = 1).
// ------------------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(kScoreThreads) void k_score_ncf(
    QueryArgs A, int64_t nE, const int64_t* __restrict__ wstart, const int32_t* __restrict__ witems,
    const int64_t* __restrict__ gstart, const int32_t* __restrict__ gq, const int64_t* __restrict__ qbase,
    const double* __restrict__ rec, int32_t* __restrict__ rel_idx, double* __restrict__ influence, int K_top,
    int32_t* __restrict__ cand_pos, double* __restrict__ cand_val) {
  static_assert(M::ncf && M::K % 4 == 0, "NCF, k a multiple of 4");
  constexpr int K = M::K, RT = kScoreRows, QB = kQueryBlock, CK = 4, H = K / 2;
  constexpr bool MASK = mask_path<M>();
  constexpr int TS = K + 1;                        // table row stride (odd: spreads the banks)
  // mask path: Tm[m2][c] = sum_e W2[c][e] W3m[e] [bit e of m2] = d1[c] / 1[z1_c > 0]
  __shared__ double Tm[MASK ? (1 << H) * TS : 1];
  if constexpr (MASK) {
    // the table (k_ncf_d1_table, once per batch) copied in with 16-B loads
    for (int t = threadIdx.x; t < (1 << H) * K / 2; t += blockDim.x) {
      const double2 v = reinterpret_cast<const double2*>(A.d1tab)[t];
      const int e = 2 * t, m2 = e / K, c = e - m2 * K;
      Tm[m2 * TS + c] = v.x;
      Tm[m2 * TS + c + 1] = v.y;
    }
    __syncthreads();
  }
  const int lane = threadIdx.x & 63;
  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int64_t n_items = wstart[nE];
  const int64_t stride = (int64_t)gridDim.x * (kScoreThreads / 64);
  const int64_t N = A.N;
  // work-item headers two stages ahead (scalar loads): the {entity, chunk, block} words of item
  // i + 2 and the list / group bounds of item i + 1 are in flight while item i is scored (most
  // yelp-ex items are short lists: the header chain was two of an item's ~four latencies)
  struct Words { int32_t g, cidx, qblk; };
  struct Bounds { int64_t p0, p1, s0, s1; };
  auto words = [&](int64_t w) {
    const int64_t wc = w < n_items ? w : n_items - 1;
    return Words{witems[3 * wc], witems[3 * wc + 1], witems[3 * wc + 2]};
  };
  auto bounds = [&](const Words& w) {
    const int sd = w.g >= A.U ? 1 : 0;
    const int32_t e = sd ? (int32_t)(w.g - A.U) : w.g;
    return Bounds{A.ptr[sd][e], A.ptr[sd][e + 1], gstart[w.g], gstart[w.g + 1]};
  };
  int64_t wi = (int64_t)blockIdx.x * (kScoreThreads / 64) + wave;
  if (wi >= n_items) return;
  Words w_cur = words(wi);
  Bounds b_cur = bounds(w_cur);
  Words w_nxt = words(wi + stride);
  for (; wi < n_items; wi += stride) {
    const Words w_n = w_nxt;
    const Bounds b_n = bounds(w_n);
    w_nxt = words(wi + 2 * stride);
    const int32_t g = w_cur.g, cidx = w_cur.cidx, qblk = w_cur.qblk;
    const int sd = g >= A.U ? 1 : 0;
    const int64_t lb = b_cur.p0 + (int64_t)cidx * kChunk;
    const int64_t rem = b_cur.p1 - lb;
    const int len = rem < kChunk ? (int)rem : kChunk;
    const int64_t gb = b_cur.s0 + (int64_t)qblk * QB;
    const int64_t gn = b_cur.s1 - gb;
    const int nq = gn < QB ? (int)gn : QB;
    w_cur = w_n;
    b_cur = b_n;

    const int32_t* __restrict__ oth = A.other[sd] + lb;
    const float* __restrict__ rat = A.rating[sd] + lb;
    const int32_t* __restrict__ rw = A.row[sd] + lb;
    const double* __restrict__ gml = A.lgm[sd] + lb;
    const int32_t* __restrict__ lmk = reinterpret_cast<const int32_t*>(A.lgm[sd]) + lb;   // mask path
    const double* __restrict__ res = A.lres + (int64_t)sd * N + lb;
    int32_t o_[RT], row_[RT], li_[RT], mk_[RT];
    float y_[RT];
    double ej[RT];
    bool ok_[RT];
#pragma unroll
    for (int r = 0; r < RT; ++r) {
      const int idx = r * 64 + lane;
      ok_[r] = idx < len;
      li_[r] = ok_[r] ? idx : 0;
      o_[r] = oth[li_[r]];
      y_[r] = rat[li_[r]];
      row_[r] = rw[li_[r]];
      ej[r] = res[li_[r]];
      mk_[r] = MASK ? lmk[li_[r]] : 0;
    }
    const float* __restrict__ T = sd == 0 ? A.t[3] : A.t[2];    // other side's gmf table
    // NQ = nq rounded up to a power of two: a static query count per path, so the
    // accumulators stay in registers without per-query exits (the padding columns
    // score copies of the last query and are never written out)
    // RTE = rows per lane actually scored: a chunk of <= 64 ratings (most lists at yelp-ex, ~24
    // ratings per user or item) runs one row per lane instead of four
    auto run = [&](auto nq_c, auto rt_c) {
      constexpr int NQ = decltype(nq_c)::value;
      constexpr int RTE = decltype(rt_c)::value;
      const double* __restrict__ xq[NQ];        // uniform: this side's record block of each query
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        const int32_t q = gq[gb + (j < nq ? j : nq - 1)];
        xq[j] = rec + (int64_t)q * M::R + 4 + sd * M::SB;
      }
      double acc[NQ][RTE];
#pragma unroll
      for (int j = 0; j < NQ; ++j)
#pragma unroll
        for (int r = 0; r < RTE; ++r) acc[j][r] = 0.0;
#pragma unroll 1
      for (int c0 = 0; c0 < K; c0 += CK) {
        double gm_[RTE][CK];
        float go_[RTE][CK];
        // scalar base per coordinate + 32-bit lane offsets (kept opaque so the compiler
        // does not strength-reduce them into 2 VGPRs per (row, coordinate) pointer)
        const double* gbase = gml + (int64_t)c0 * N;
        if constexpr (!MASK) asm volatile("" : "+s"(gbase));
#pragma unroll
        for (int r = 0; r < RTE; ++r) {
          if constexpr (MASK) {
            // d1 of rating r at coordinates c0 .. c0 + 3 (mask path; x_mlp is y = W1^T x here)
            const double* __restrict__ Tr = Tm + (mk_[r] >> K) * TS + c0;
#pragma unroll
            for (int cc = 0; cc < CK; ++cc) gm_[r][cc] = (mk_[r] >> (c0 + cc)) & 1 ? Tr[cc] : 0.0;
          } else {
#pragma unroll
            for (int cc = 0; cc < CK; ++cc) gm_[r][cc] = gbase[(int64_t)cc * N + li_[r]];
          }
          const float4 t = *reinterpret_cast<const float4*>(T + (int64_t)o_[r] * K + c0);
          go_[r][0] = t.x; go_[r][1] = t.y; go_[r][2] = t.z; go_[r][3] = t.w;
        }
#pragma unroll
        for (int j = 0; j < NQ; ++j) {
#pragma unroll
          for (int c2 = 0; c2 < CK / 2; ++c2) {
            // scalar loads: x_mlp and W3g * x_gmf as SGPR operands (no LDS)
            const double ax = xq[j][c0 + 2 * c2], ay = xq[j][c0 + 2 * c2 + 1];
            const double bx = xq[j][K + c0 + 2 * c2], by = xq[j][K + c0 + 2 * c2 + 1];
#pragma unroll
            for (int r = 0; r < RTE; ++r) {
              acc[j][r] = fma(ax, gm_[r][2 * c2], acc[j][r]);
              acc[j][r] = fma(ay, gm_[r][2 * c2 + 1], acc[j][r]);
              acc[j][r] = fma(bx, (double)go_[r][2 * c2], acc[j][r]);
              acc[j][r] = fma(by, (double)go_[r][2 * c2 + 1], acc[j][r]);
            }
          }
        }
      }
#pragma unroll
      for (int j = 0; j < NQ; ++j) {
        if (j >= nq) continue;   // padding columns (copies of the last query)
        const int32_t q = gq[gb + j];
        const double* __restrict__ Rj = rec + (int64_t)q * M::R;
        const double inv_n = Rj[0], cq = Rj[1], xv = Rj[2], rhat_ui = Rj[3];
        const double dup_o = xq[j][2 * K];
        const int64_t* __restrict__ qb = qbase + 4 * (int64_t)q;
        const int64_t obj = qb[sd] + (int64_t)cidx * kChunk, cbj = qb[2 + sd] + cidx;
        const int64_t poj = sd ? qb[1] - qb[0] : 0;   // |R_u| precedes item-side positions
        double la[RTE], lv[RTE];
        int lp[RTE];
#pragma unroll
        for (int r = 0; r < RTE; ++r) {
          double ee = ej[r], ss = acc[j][r];
          if ((double)o_[r] == dup_o) { ee = rhat_ui - (double)y_[r]; ss = xv; }
          const double infl = (2.0 * ee * ss + cq) * inv_n;
          const int idx = r * 64 + lane;
          if (ok_[r]) {
            if (influence) __builtin_nontemporal_store(infl, influence + obj + idx);
            if (rel_idx) __builtin_nontemporal_store(row_[r], rel_idx + obj + idx);
          }
          lp[r] = ok_[r] ? cidx * kChunk + idx : -1;
          la[r] = ok_[r] ? topk_key(infl) : -2.0;
          lv[r] = infl;
        }
        if (K_top > 0) {
          double pa = INFINITY;
          int pp = -1;
          for (int t = 0; t < K_top; ++t) {
            double ba = -2.0, bv = 0.0;
            int bp = 0x7fffffff;
#pragma unroll
            for (int r = 0; r < RTE; ++r)
              if (lp[r] >= 0 && better(pa, pp, la[r], lp[r]) && better(la[r], lp[r], ba, bp)) {
                ba = la[r]; bp = lp[r]; bv = lv[r];
              }
            wave_best(ba, bp, bv);
            if (lane == 0) {
              const bool okk = ba > -1.5;
              const int64_t slot = cbj * K_top + t;
              cand_pos[slot] = okk ? (int32_t)(bp + poj) : -1;
              cand_val[slot] = okk ? bv : NAN;
            }
            pa = ba;
            pp = bp;
          }
        }
      }
    };
    auto run_q = [&](auto rt_c) {
      if (nq <= 1) run(std::integral_constant<int, 1>{}, rt_c);
      else if (nq <= 2) run(std::integral_constant<int, 2>{}, rt_c);
      else if (nq <= 4) run(std::integral_constant<int, 4>{}, rt_c);
      else run(std::integral_constant<int, QB>{}, rt_c);
    };
    if (len <= 64) run_q(std::integral_constant<int, 1>{});
    else run_q(std::integral_constant<int, RT>{});
    __builtin_amdgcn_wave_barrier();
  }
}

// Merge the chunk candidates of every query (one wave per query).
__global__ __launch_bounds__(64) void k_topk_merge(const int32_t* __restrict__ qu, const int32_t* __restrict__ qi,
                                                   int64_t Q, const int64_t* __restrict__ coff, int K, int spc,
                                                   const int32_t* __restrict__ cand_pos,
                                                   const double* __restrict__ cand_val,
                                                   const int64_t* __restrict__ uptr, const int32_t* __restrict__ urow,
                                                   const int64_t* __restrict__ iptr, const int32_t* __restrict__ irow,
                                                   int64_t U, int64_t I, int64_t* __restrict__ topk_pos,
                                                   int64_t* __restrict__ topk_idx, double* __restrict__ topk_val) {
  const int64_t q = blockIdx.x;
  if (q >= Q) return;
  const int lane = threadIdx.x;
  const int64_t cb = coff[q] * spc * K, ce = coff[q + 1] * spc * K;
  const int32_t u = qu[q], i = qi[q];
  const bool ok_id = (u >= 0 && u < U && i >= 0 && i < I);
  const int64_t ub = ok_id ? uptr[u] : 0, du = ok_id ? uptr[u + 1] - ub : 0, ib = ok_id ? iptr[i] : 0;
  double pa = INFINITY;
  int pp = -1;
  for (int t = 0; t < K; ++t) {
    double ba = -2.0, bv = 0.0;
    int bp = 0x7fffffff;
    for (int64_t c = cb + lane; c < ce; c += 64) {
      const int p = cand_pos[c];
      if (p < 0) continue;
      const double vv = cand_val[c];
      const double a = topk_key(vv);
      if (better(pa, pp, a, p) && better(a, p, ba, bp)) { ba = a; bp = p; bv = vv; }
    }
    wave_best(ba, bp, bv);
    if (lane == 0) {
      const bool ok = ba > -1.5;
      topk_pos[q * K + t] = ok ? bp : -1;
      topk_idx[q * K + t] = ok ? (int64_t)(bp < du ? urow[ub + bp] : irow[ib + (bp - du)]) : -1;
      topk_val[q * K + t] = ok ? bv : NAN;
    }
    pa = ba;
    pp = bp;
  }
}

// Small K: one THREAD per query walks its chunks' candidates K times (a query has a few to a
// few hundred candidate slots; a wave per query mostly idles at K = 1).  Same order and
// output as k_topk_merge.
__global__ __launch_bounds__(256) void k_topk_merge_thread(
    const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t Q, const int64_t* __restrict__ coff,
    int K, int spc, const int32_t* __restrict__ cand_pos, const double* __restrict__ cand_val,
    const int64_t* __restrict__ uptr, const int32_t* __restrict__ urow, const int64_t* __restrict__ iptr,
    const int32_t* __restrict__ irow, int64_t U, int64_t I, int64_t* __restrict__ topk_pos,
    int64_t* __restrict__ topk_idx, double* __restrict__ topk_val) {
  const int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (q >= Q) return;
  const int64_t cb = coff[q] * spc * K, ce = coff[q + 1] * spc * K;
  const int32_t u = qu[q], i = qi[q];
  const bool ok_id = (u >= 0 && u < U && i >= 0 && i < I);
  const int64_t ub = ok_id ? uptr[u] : 0, du = ok_id ? uptr[u + 1] - ub : 0, ib = ok_id ? iptr[i] : 0;
  double pa = INFINITY;
  int pp = -1;
  for (int t = 0; t < K; ++t) {
    double ba = -2.0, bv = 0.0;
    int bp = 0x7fffffff;
    // both words of a slot loaded unconditionally (empty slots hold -1 / NaN) and 4 slots
    // per round, so the candidate reads are one round trip per 4 slots, not two per slot
    int64_t c = cb;
    for (; c + 4 <= ce; c += 4) {
      int p4[4];
      double v4[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) { p4[j] = cand_pos[c + j]; v4[j] = cand_val[c + j]; }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const double a = topk_key(v4[j]);
        if (p4[j] >= 0 && better(pa, pp, a, p4[j]) && better(a, p4[j], ba, bp)) { ba = a; bp = p4[j]; bv = v4[j]; }
      }
    }
    for (; c < ce; ++c) {
      const int p = cand_pos[c];
      const double vv = cand_val[c];
      const double a = topk_key(vv);
      if (p >= 0 && better(pa, pp, a, p) && better(a, p, ba, bp)) { ba = a; bp = p; bv = vv; }
    }
    const bool ok = ba > -1.5;
    topk_pos[q * K + t] = ok ? bp : -1;
    topk_idx[q * K + t] = ok ? (int64_t)(bp < du ? urow[ub + bp] : irow[ib + (bp - du)]) : -1;
    topk_val[q * K + t] = ok ? bv : NAN;
    pa = ba;
    pp = bp;
  }
}

// ------------------------------------------------------------------------------------
// host-side dispatch
// ------------------------------------------------------------------------------------
QueryArgs make_args(fia_ctx* c, const int32_t* qu, const int32_t* qi) {
  QueryArgs A{};
  A.qu = qu;
  A.qi = qi;
  A.U = c->p.U;
  A.I = c->p.I;
  for (int s = 0; s < 2; ++s) {
    A.ptr[s] = c->idx.side[s].ptr.as<int64_t>();
    A.row[s] = c->idx.side[s].row.as<int32_t>();
    A.other[s] = c->idx.side[s].other.as<int32_t>();
    A.rating[s] = c->idx.side[s].rating.as<float>();
    A.gram[s] = c->gram[s].as<double>();
    A.l1[s] = c->l1[s].as<double>();
  }
  for (int t = 0; t < 10; ++t) A.t[t] = c->p.t[t];
  A.wd = c->p.wd;
  A.damping = c->p.damping;
  A.pairs.key = c->idx.pkey.as<unsigned long long>();
  A.pairs.cnt = c->idx.pcnt.as<int32_t>();
  A.pairs.sum = c->idx.psum.as<double>();
  A.pairs.mask = (unsigned long long)(c->idx.pcap - 1);
  A.lgm[0] = c->gm[0].as<double>();
  A.lgm[1] = c->gm[1].as<double>();
  A.lres = c->resid.as<double>();
  A.N = c->idx.N;
  return A;
}

// MF k = 16: a quad of lanes per side system (k_solve_quad); MF k = 8: a thread per system
template <class M>
constexpr bool use_quad_solve() {
  return !M::ncf && M::K == 16;
}
template <class M>
constexpr bool use_tps() {
  return !M::ncf && M::Ds <= 17 && !use_quad_solve<M>();
}

// side systems on 16x16 tiles: NCF (Ds = 2k) and MF k >= 32 (k coordinates + the bias)
template <class M>
constexpr bool use_tile_solve() {
  return !use_tps<M>() && !use_quad_solve<M>() && (M::ncf ? M::Ds : M::K) % 16 == 0 &&
         (M::ncf ? M::Ds : M::K) <= 64;
}

// NCF k <= 16: both side blocks in one wave, a column per lane (k_solve_col)
template <class M>
constexpr bool use_col_solve() {
  return M::ncf && 2 * M::Ds <= 64;
}

// one side-system solve per model: MF k <= 16 k_solve_tps, NCF k = 16 k_solve_rows, NCF k = 8
// k_solve_col, MF k in {32, 64} and NCF k = 32 k_solve_tile
template <class M>
constexpr bool solve_covered() {
  return use_quad_solve<M>() || use_tps<M>() || pair_layout<M>() || use_col_solve<M>() || use_tile_solve<M>();
}

// MF k <= 16 item runs: slice cost target (descriptor cost units per one-wave slice; ml-1m-ex
// same-box A/B, scoring us -- round 4: 8 -> 69.4, 16 -> 68.6, 32 -> 73.5, 64 -> 78.6; round 5
// (this kernel): 4 -> 62.0, 8 -> 58.0-58.6, 16 -> 58.8; chunks of 64 / 192 / 256 ratings at
// 8: 66.3 / 62.0 / 85.8 vs 128; runs of <= 32 queries: 62.6)
constexpr int kRunLambda = 8;

// MF k <= 16: the Gram stream (its descriptors carry the entity in 24 bits)
template <class M>
bool use_gram_stream(const int64_t (&n_ent)[2]) {
  // (and a table's bytes in a 32-bit buffer range)
  return !M::ncf && M::K <= 16 && n_ent[0] < (1 << 23) && n_ent[1] < (1 << 23);
}

template <class M>
hipError_t prepare_impl(fia_ctx* c, hipStream_t s, const uint8_t* mark) {
  constexpr int Ds = M::Ds, GS = Ds * (Ds + 1) / 2, K = M::K;
  const int64_t n_ent[2] = {c->p.U, c->p.I};
  for (int sd = 0; sd < 2; ++sd) FIA_HIP_TRY(c->gram[sd].reserve(sizeof(double) * (size_t)(n_ent[sd] * ((GS + 1) & ~1) + 1), s));
  if constexpr (M::ncf) {
    for (int sd = 0; sd < 2; ++sd) {
      FIA_HIP_TRY(c->l1[sd].reserve(sizeof(double) * (size_t)(n_ent[sd] * K + 1), s));
      const int64_t tot = n_ent[sd] * K;
      if (tot > 0) {
        hipLaunchKernelGGL(k_ncf_l1<K>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, c->p.t[sd],
                           c->p.t[4], sd * K, n_ent[sd], c->l1[sd].as<double>());
        FIA_HIP_TRY(hipGetLastError());
      }
    }
    if (s == c->aux && c->l1_ev) {       // on the aux stream: the query prologue may start here
      FIA_HIP_TRY(hipEventRecord(c->l1_ev, s));
      c->l1_pending = true;
    }
  }
  constexpr int GSP = (GS + 1) & ~1;
  // the slice lists of the per-slice Gram kernels (k_ncf_gram_rows, k_gram_mf_mfma); the MF
  // k <= 16 Gram stream cuts its own sub-batches (build_gram_stream) and needs neither these
  // lists nor their partial-Gram slots
  const bool stream = use_gram_stream<M>(n_ent);
  // Gram slice length: short slices for parallelism, long enough that the partial Grams
  // of split lists (GSP doubles each) stay a few bytes per rating (MI355X: ml-1m-ex MF k=16
  // best at 256, 20M MF k=64 loses 30% at 256 vs 512)
  if (!stream) {
    int64_t want = 256;
    while (!M::ncf && want < 4096 && want < GSP) want *= 2;   // NCF: 256 (16 slabs per item)
    if (c->idx.gchunk != want) FIA_HIP_TRY(build_gram_lists(c, want, s));
  }
  const Index& X = c->idx;
  for (int sd = 0; sd < 2 && !stream; ++sd)
    if (X.n_gslots[sd] > 0) FIA_HIP_TRY(c->gpart[sd].reserve(sizeof(double) * (size_t)(X.n_gslots[sd] * GSP), s));
  GramSides G{};
  for (int sd = 0; sd < 2; ++sd) {
    G.n_items[sd] = n_ent[sd] > 0 ? X.n_gitems[sd] : 0;
    G.items[sd] = X.gitems[sd].as<int32_t>();
    G.ptr[sd] = X.side[sd].ptr.as<int64_t>();
    G.other[sd] = X.side[sd].other.as<int32_t>();
    G.emb_other[sd] = M::ncf ? c->p.t[sd == 0 ? 3 : 2] : c->p.t[sd == 0 ? 1 : 0];   // NCF: gmf tables
    G.gram[sd] = c->gram[sd].as<double>();
    G.part[sd] = c->gpart[sd].as<double>();
    G.lgm[sd] = c->gm[sd].as<double>();
  }
  G.W3 = c->p.t[8];
  G.N = X.N;
  G.mark = mark;
  G.moff[0] = 0;
  G.moff[1] = n_ent[0];
  if constexpr (M::ncf) {
    // per list position of each side: g_mlp (coordinate-major) and e, with the Grams
    const int64_t N = X.N;
    // g_mlp coordinate-major [k][N], or (mask path) the ReLU masks int32 [N]
    const size_t per = mask_path<M>() ? sizeof(int32_t) * (size_t)(N + 2) : sizeof(double) * (size_t)(N * K + 1);
    for (int sd = 0; sd < 2; ++sd) FIA_HIP_TRY(c->gm[sd].reserve(per, s));
    FIA_HIP_TRY(c->resid.reserve(sizeof(double) * (size_t)(2 * N + 1), s));
    for (int sd = 0; sd < 2; ++sd) G.lgm[sd] = c->gm[sd].as<double>();
    const int64_t n_all = G.n_items[0] + G.n_items[1];
    if (n_all > 0) {
      // persistent: the per-lane weight operands are loaded once per wave.  8 waves per CU fill
      // every CU (2 per SIMD at its registers); when other contexts share the GPU (batches in
      // flight) 6, so their kernels run beside the pass instead of after it (yelp-ex, 2 in
      // flight, same box: 102.1 -> 106.0-106.4 M q/s; one context alone: 92.5 at 8, 85.9 at 6)
      const int per_cu = live_contexts(c->device) > 1 ? 6 : 8;
      const int64_t cap = (int64_t)(c->num_cus > 0 ? c->num_cus : 256) * per_cu;
      const int64_t grid = n_all < cap ? n_all : cap;
      hipLaunchKernelGGL(k_ncf_gram_rows<M>, dim3((unsigned)grid), dim3(64), 0, s, G, c->p.t[4], c->p.t[5],
                         c->p.t[6], c->p.t[7], c->p.t[9], c->l1[0].as<double>(), c->l1[1].as<double>(),
                         X.side[0].rating.as<float>(), X.side[1].rating.as<float>(), c->resid.as<double>());
      FIA_HIP_TRY(hipGetLastError());
    }
  } else if (stream) {
    // MF k <= 16: the Gram stream (both sides, one launch), then the partial slices combined
    FIA_HIP_TRY(build_gram_stream(c, K, s));
    for (int sd = 0; sd < 2; ++sd)
      if (X.n_gsslots[sd] > 0) FIA_HIP_TRY(c->gpart[sd].reserve(sizeof(double) * (size_t)(X.n_gsslots[sd] * GSP), s));
    GramStreamArgs GT{};
    GT.desc = X.gsdesc.as<int2>();
    GT.ids = X.gsids.as<uint32_t>();
    GT.wave = X.gswave.as<int32_t>();
    GT.n_waves = X.n_gsw;
    for (int sd = 0; sd < 2; ++sd) {
      GT.emb_other[sd] = c->p.t[sd == 0 ? 1 : 0];
      GT.bytes_other[sd] = (uint32_t)(n_ent[1 - sd] * K * (int64_t)sizeof(float));
      GT.gram[sd] = c->gram[sd].as<double>();
      GT.part[sd] = c->gpart[sd].as<double>();
    }
    GT.mark = mark;
    GT.moff[0] = 0;
    GT.moff[1] = n_ent[0];
    if (X.n_gsw > 0) FIA_HIP_TRY(launch_gram_mf_stream(M::K, GT, s));
    const int64_t nc0 = X.n_gscomb[0], nc1 = X.n_gscomb[1];
    if (nc0 + nc1 > 0) {
      hipLaunchKernelGGL(k_gram_combine, dim3((unsigned)(nc0 + nc1)), dim3(256), 0, s, nc0, X.gscomb[0].as<int32_t>(),
                         c->gpart[0].as<double>(), c->gram[0].as<double>(), nc1, X.gscomb[1].as<int32_t>(),
                         c->gpart[1].as<double>(), c->gram[1].as<double>(), GS, GSP, mark, n_ent[0]);
      FIA_HIP_TRY(hipGetLastError());
    }
    return hipSuccess;
  } else {
    if constexpr (K == 32 || K == 64) {
      // list-ordered residuals of both sides for k_score_mf_mfma ([0, N) users, [N, 2N) items),
      // written by the Gram pass for every list position of a cached entity
      FIA_HIP_TRY(c->resid.reserve(sizeof(double) * (size_t)(2 * X.N + 1), s));
      for (int sd = 0; sd < 2; ++sd) {
        G.emb_self[sd] = c->p.t[sd];
        G.rating[sd] = X.side[sd].rating.as<float>();
        G.bias[sd] = c->p.t[2 + sd];
      }
      G.gb = c->p.t[4];
      G.lres = c->resid.as<double>();
    }
    if (G.n_items[0] + G.n_items[1] > 0) {
      hipLaunchKernelGGL(k_gram_mf_mfma<M>, dim3((unsigned)(G.n_items[0] + G.n_items[1])), dim3(64), 0, s, G);
      FIA_HIP_TRY(hipGetLastError());
    }
  }
  const int64_t nc0 = n_ent[0] > 0 ? X.n_gcomb[0] : 0, nc1 = n_ent[1] > 0 ? X.n_gcomb[1] : 0;
  if (nc0 + nc1 > 0) {
    hipLaunchKernelGGL(k_gram_combine, dim3((unsigned)(nc0 + nc1)), dim3(256), 0, s, nc0, X.gcomb[0].as<int32_t>(),
                       c->gpart[0].as<double>(), c->gram[0].as<double>(), nc1, X.gcomb[1].as<int32_t>(),
                       c->gpart[1].as<double>(), c->gram[1].as<double>(), GS, GSP, mark, n_ent[0]);
    FIA_HIP_TRY(hipGetLastError());
  }
  return hipSuccess;
}

template <class M>
hipError_t query_impl(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                      int64_t max_chunks, int32_t* rel_idx, double* influence, double* x_out, int K,
                      int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                      const double* x_in) {
  // One scoring schedule per (model, k, K) (measured on MI355X, profiles/): k <= 16 item runs
  // (MF k_score_mf_runs, NCF k_score_ncf_runs: per-query chunks sharing the item's list); MF
  // k in {32, 64} entity-shared, on f64 MFMA for K <= 1 (k_score_mf_mfma, query blocks of 16)
  // and on VALU otherwise (k_score_grouped_mf); NCF k = 32 entity-shared (k_score_ncf)
  constexpr bool grouped = M::ncf ? !mask_path<M>() : M::K >= 32;
  constexpr bool mfma_ok = !M::ncf && (M::K == 32 || M::K == 64);
  const bool use_mfma = mfma_ok && K <= 1;
  // (the MFMA kernel's work item is a group of kWgBlocks query blocks, one per wave)
  const int qblock = use_mfma ? kMfmaQB * kWgBlocks : query_block<M>();
  constexpr bool runs = !grouped;
  constexpr int spc = 1;      // candidate slot sets per chunk
  static_assert(solve_covered<M>(), "every small-k model has a side-system solve");
  FIA_HIP_TRY(c->rec.reserve(sizeof(double) * (size_t)(Q * M::R + 1), s));
  if (K > 0) {
    FIA_HIP_TRY(c->cand_pos.reserve(sizeof(int32_t) * (size_t)((max_chunks + 1) * K * spc), s));
    FIA_HIP_TRY(c->cand_val.reserve(sizeof(double) * (size_t)((max_chunks + 1) * K * spc), s));
  }
  QueryArgs A = make_args(c, qu, qi);
  const int64_t nE = c->idx.U + c->idx.I;
  // every (entity chunk, query block) item covers >= 1 per-query chunk
  const int64_t max_items = max_chunks;
  // the queries whose test pair is a train row are listed in `coupled` {count, q...} by the
  // solve and finished full-D; the chunk scan zeroes the count
  FIA_HIP_TRY(c->coupled.reserve(sizeof(int32_t) * (size_t)(Q + 1), s));
  // MF k <= 16: the chunk phase is the one scan kernel and the solve phase the side-system solve
  // + the coupled solve, so their events are stamped by those kernels' dispatches (a marker
  // packet per event idled the GPU ~5 us: RQ2's single query)
  constexpr bool ext_phases = runs && !M::ncf && use_quad_solve<M>();
  PhaseSpan cspan;
  if (ext_phases) {
    cspan = phase_span(c, 4);
    c->scan_ev[0] = cspan.a;
    c->scan_ev[1] = cspan.b;
  } else {
    phase_begin(c, 4, s);
  }
  // MF k <= 16 item runs: one wave per equal-cost slice of the descriptor list (descriptor
  // costs vary ~10x: a static stride over descriptors left waves idle for half the kernel);
  // the slice count is known on the device only -- the grid is its bound (total cost <=
  // kRunUserCost per descriptor slot), the surplus waves exit at once
  constexpr int64_t lam = kRunLambda;
  const int64_t runs_grid = (kRunUserCost * (max_chunks + 1)) / lam + 2;
  {
    const hipError_t eb = build_chunks(c, Q, qu, qi, offsets, max_chunks, grouped, s, c->coupled.as<int32_t>(), runs,
                                       (int)lam, M::ncf ? kNcfRunChunk : kRunChunk);
    c->scan_ev[0] = c->scan_ev[1] = nullptr;
    FIA_HIP_TRY(eb);
  }
  if (grouped) FIA_HIP_TRY(build_groups(c, Q, qu, qi, offsets, max_items, qblock, s, use_mfma ? kMfmaCPI : 1));
  // the query-side work that needs no Gram cache, ahead of the join with a pending prepare:
  // NCF k = 16 the per-query MLP prologue (after the layer-1 rows), k <= 16 the d1 table
  // (timed with the chunk lists: the solve phase starts after the join)
  if constexpr (pair_layout<M>()) {
    if (Q > 0 && !x_in) {
      FIA_HIP_TRY(join_l1(c, s));
      FIA_HIP_TRY(c->qwork.reserve(sizeof(double) * (size_t)(Q * qpro_stride<M>() + 1), s));
      hipLaunchKernelGGL(k_ncf_query_pro<M>, dim3((unsigned)((Q + 63) / 64)), dim3(256), 0, s, A, Q,
                         c->qwork.as<double>());
      FIA_HIP_TRY(hipGetLastError());
    }
  }
  if constexpr (mask_path<M>()) {
    if (Q > 0) {
      constexpr int NT = (1 << (M::K / 2)) * M::K;
      FIA_HIP_TRY(c->d1tab.reserve(sizeof(double) * NT, s));
      hipLaunchKernelGGL(k_ncf_d1_table<M>, dim3((unsigned)((NT + 255) / 256)), dim3(256), 0, s, c->p.t[6], c->p.t[8],
                         c->d1tab.as<double>());
      FIA_HIP_TRY(hipGetLastError());
      A.d1tab = c->d1tab.as<double>();
    }
  }
  if (!ext_phases) phase_end(c, 4, s);
  FIA_HIP_TRY(join_prepare(c, s));     // the Gram caches (and NCF rows) of a pending fia_prepare
  const bool ext_solve = ext_phases && Q > 0 && !x_in;
  PhaseSpan sspan;
  if (ext_solve) sspan = phase_span(c, 1);
  else phase_begin(c, 1, s);
  if (x_in && Q > 0) {
    // a given inverse HVP: records straight from it, no solve (fia_query_batch_x)
    const int64_t g1 = Q < 8192 ? Q : 8192;
    hipLaunchKernelGGL(k_record_x<M>, dim3((unsigned)g1), dim3(kSolveThreads), 0, s, A, Q, x_in, c->rec.as<double>(),
                       x_out);
    FIA_HIP_TRY(hipGetLastError());
  }
  // non-coupled queries: thread-per-system (MF k <= 16) or column-parallel blocks
  if (Q > 0 && !x_in) {
    if constexpr (use_quad_solve<M>()) {
      hipExtLaunchKernelGGL(k_solve_quad<M>, dim3((unsigned)((Q + 7) / 8)), dim3(64), 0, s, sspan.a, (hipEvent_t) nullptr, 0, A, Q,
                            c->rec.as<double>(), x_out, c->coupled.as<int32_t>());
    } else if constexpr (use_tps<M>()) {
      hipLaunchKernelGGL(k_solve_tps<M>, dim3((unsigned)((2 * Q + 63) / 64)), dim3(64), 0, s, A, Q,
                         c->rec.as<double>(), x_out, c->coupled.as<int32_t>());
    } else if constexpr (pair_layout<M>()) {
      hipLaunchKernelGGL(k_solve_rows<M>, dim3((unsigned)((Q + 1) / 2)), dim3(64), 0, s, A, Q,
                         (const double*)c->qwork.as<double>(), c->rec.as<double>(), x_out, c->coupled.as<int32_t>());
    } else if constexpr (use_col_solve<M>()) {
      const int64_t cap = (int64_t)(c->num_cus > 0 ? c->num_cus : 256) * 16;
      constexpr int QW = 32 / M::K;             // queries per wave
      const int64_t need = (Q + QW - 1) / QW;
      const int64_t g1 = need < cap ? need : cap;   // persistent: NCF weights staged once per block
      hipLaunchKernelGGL(k_solve_col<M>, dim3((unsigned)g1), dim3(64), 0, s, A, Q, c->rec.as<double>(), x_out,
                         c->coupled.as<int32_t>());
    } else {
      const int64_t cap = (int64_t)(c->num_cus > 0 ? c->num_cus : 256) * 8;
      const int64_t g1 = Q < cap ? Q : cap;     // persistent: NCF weights staged once per block
      hipLaunchKernelGGL(k_solve_tile<M>, dim3((unsigned)g1), dim3(128), 0, s, A, Q, c->rec.as<double>(), x_out,
                         c->coupled.as<int32_t>());
    }
    FIA_HIP_TRY(hipGetLastError());
    // usually no coupled query: a small grid that exits (a full grid for the large full-D
    // systems of k >= 32, should many test pairs be train rows).  (Folding this into the last
    // workgroup of k_solve_tps -- an atomic finish count -- made that kernel 14 us slower at
    // ml-1m-ex: the full-D solve's LDS and registers in every workgroup)
    const int64_t gc = M::K <= 16 ? 64 : 256;
    const int64_t g2 = Q < gc ? Q : gc;
    hipExtLaunchKernelGGL(k_solve<M>, dim3((unsigned)g2), dim3(kSolveThreads), 0, s, (hipEvent_t) nullptr,
                          sspan.b, 0, A, Q, c->rec.as<double>(), x_out, (const int32_t*)c->coupled.as<int32_t>());
  }
  if constexpr (mask_path<M>()) {
    if (Q > 0) {       // the records' MLP block -> y = W1_side^T x_mlp for k_score_ncf
      hipLaunchKernelGGL(k_ncf_rec_y<M>, dim3((unsigned)((2 * Q + 255) / 256)), dim3(256), 0, s, Q, c->p.t[4],
                         c->rec.as<double>());
    }
  }
  FIA_HIP_TRY(hipGetLastError());
  if (!ext_solve) phase_end(c, 1, s);
  int64_t grid = (max_items + 3) / 4;            // 4 waves (work items) per block
  if (grid < 1) grid = 1;
  // grid cap (measured): NCF 1024 workgroups (yelp-ex score 0.314 -> 0.290 ms), MF 8192
  const int64_t gcap = M::ncf ? 1024 : 8192;
  if (grid > gcap) grid = gcap;
  if (runs) grid = runs_grid;
  // the MFMA kernel: one work item per workgroup (grid-stride)
  if (use_mfma) grid = max_items < 8192 ? (max_items > 0 ? max_items : 1) : 8192;
  const PhaseSpan span = phase_span(c, 2);
  if (grouped) {
    if constexpr (M::ncf)
      hipExtLaunchKernelGGL(k_score_ncf<M>, dim3((unsigned)grid), dim3(kScoreThreads), 0, s, span.a, span.b, 0, A, nE,
                         c->wstart.as<int64_t>(), c->witems.as<int32_t>(), c->gstart.as<int64_t>(),
                         c->gq.as<int32_t>(), c->qbase.as<int64_t>(), c->rec.as<double>(), rel_idx, influence, K,
                         c->cand_pos.as<int32_t>(), c->cand_val.as<double>());
    else {
      if constexpr (mfma_ok) {
        if (use_mfma) {
          FIA_HIP_TRY(launch_score_mf_mfma(M::K, rel_idx && influence, grid, s, span, A, nE, c->wstart.as<int64_t>(),
                                           c->witems.as<int32_t>(), c->gstart.as<int64_t>(), c->gq.as<int32_t>(),
                                           c->qbase.as<int64_t>(), c->rec.as<double>(), rel_idx, influence, K,
                                           c->cand_pos.as<int32_t>(), c->cand_val.as<double>()));
          goto topk;
        }
      }
      hipExtLaunchKernelGGL(k_score_grouped_mf<M>, dim3((unsigned)grid), dim3(kScoreThreads), 0, s, span.a, span.b, 0,
                            A, nE,
                         c->wstart.as<int64_t>(), c->witems.as<int32_t>(), c->gstart.as<int64_t>(),
                         c->gq.as<int32_t>(), c->qbase.as<int64_t>(), c->rec.as<double>(), rel_idx, influence, K,
                         c->cand_pos.as<int32_t>(), c->cand_val.as<double>());
    }
  } else {
    // k <= 16: item runs
    if constexpr (runs && !M::ncf)
      FIA_HIP_TRY(launch_score_mf_runs(M::K, grid, s, A, Q, c->cdesc.as<ChunkDesc>(), c->qbase.as<int64_t>(),
                                       c->slices.as<int32_t>(), c->rec.as<double>(), rel_idx, influence, K,
                                       c->cand_pos.as<int32_t>(), c->cand_val.as<double>(), span));
    if constexpr (runs && M::ncf)
      FIA_HIP_TRY(launch_score_ncf_runs(M::K, grid, s, A, Q, c->cdesc.as<ChunkDesc>(), c->qbase.as<int64_t>(),
                                        c->slices.as<int32_t>(), c->rec.as<double>(), rel_idx, influence, K,
                                        c->cand_pos.as<int32_t>(), c->cand_val.as<double>(), span));
  }
  FIA_HIP_TRY(hipGetLastError());
topk:
  if (K > 0 && Q > 0) {
    phase_begin(c, 3, s);
    FIA_HIP_TRY(launch_topk_merge(c, Q, qu, qi, K, spc, topk_pos, topk_idx, topk_val, s, max_chunks));
    phase_end(c, 3, s);
  }
  return hipSuccess;
}

}  // namespace

#define FIA_MODEL_CASES(X) \
  X(FIA_MODEL_MF, 8, MFm<8>) X(FIA_MODEL_MF, 16, MFm<16>) X(FIA_MODEL_MF, 32, MFm<32>) \
  X(FIA_MODEL_MF, 64, MFm<64>) X(FIA_MODEL_NCF, 8, NCFm<8>) X(FIA_MODEL_NCF, 16, NCFm<16>) \
  X(FIA_MODEL_NCF, 32, NCFm<32>)

bool model_supported(int model, int k) {
#define X(m, kk, T) if (model == m && k == kk) return true;
  FIA_MODEL_CASES(X)
#undef X
  return big_supported(model, k);
}

hipError_t launch_topk_merge(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int K, int spc,
                             int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s,
                             int64_t max_chunks) {
  if (K <= 0 || Q <= 0) return hipSuccess;
  // a thread per query while the queries have few chunks (<= 16 on average: ml-1m-ex,
  // yelp-ex); a wave per query over long candidate lists (20M: ~170 chunks per query)
  if (K <= 4 && max_chunks <= 16 * Q) {
    hipLaunchKernelGGL(k_topk_merge_thread, dim3((unsigned)((Q + 255) / 256)), dim3(256), 0, s, qu, qi, Q,
                       c->coff.as<int64_t>(), K, spc, c->cand_pos.as<int32_t>(), c->cand_val.as<double>(),
                       c->idx.side[0].ptr.as<int64_t>(), c->idx.side[0].row.as<int32_t>(),
                       c->idx.side[1].ptr.as<int64_t>(), c->idx.side[1].row.as<int32_t>(), c->p.U, c->p.I, topk_pos,
                       topk_idx, topk_val);
    return hipGetLastError();
  }
  hipLaunchKernelGGL(k_topk_merge, dim3((unsigned)Q), dim3(64), 0, s, qu, qi, Q, c->coff.as<int64_t>(), K, spc,
                     c->cand_pos.as<int32_t>(), c->cand_val.as<double>(), c->idx.side[0].ptr.as<int64_t>(),
                     c->idx.side[0].row.as<int32_t>(), c->idx.side[1].ptr.as<int64_t>(),
                     c->idx.side[1].row.as<int32_t>(), c->p.U, c->p.I, topk_pos, topk_idx, topk_val);
  return hipGetLastError();
}

int model_num_params(int model, int k) {
  if (model == FIA_MODEL_MF) return 2 * k + 2;
  if (model == FIA_MODEL_NCF) return 4 * k;
  return 0;
}

hipError_t prepare_model(fia_ctx* c, hipStream_t s, bool& unsupported) {
  unsupported = false;
  c->subset = false;
  c->small_subset = false;
#define X(m, kk, T) if (c->p.model == m && c->p.k == kk) return prepare_impl<T>(c, s, nullptr);
  FIA_MODEL_CASES(X)
#undef X
  if (big_supported(c->p.model, c->p.k)) return prepare_big(c, 0, nullptr, nullptr, s);
  unsupported = true;
  return hipSuccess;
}

// fia_prepare_for, small k: the queries' users and items are marked on the device (no host
// round trip) and only their Gram caches (NCF: and per-position rows) are built; the cover
// check of later fia_count_related calls reads the same marks
__global__ void k_mark_small(int64_t Q, const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t U,
                             int64_t I, uint8_t* __restrict__ mark) {
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = qu[q], i = qi[q];
    if (u >= 0 && u < U && i >= 0 && i < I) {
      mark[u] = 1;
      mark[U + i] = 1;
    }
  }
}

__global__ void k_check_mark(int64_t Q, const int32_t* __restrict__ qu, const int32_t* __restrict__ qi, int64_t U,
                             int64_t I, const uint8_t* __restrict__ mark, int32_t* __restrict__ flag) {
  int bad = 0;
  for (int64_t q = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; q < Q; q += (int64_t)gridDim.x * blockDim.x) {
    const int32_t u = qu[q], i = qi[q];
    if (u >= 0 && u < U && i >= 0 && i < I) bad |= !mark[u] || !mark[U + i];
  }
  if (__any(bad) && (threadIdx.x & 63) == 0) atomicOr(flag, 1);
}

hipError_t prepare_model_for(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, hipStream_t s, hipStream_t ps,
                             bool& unsupported, bool mark_only) {
  unsupported = false;
  const int64_t U = c->p.U, I = c->p.I;
  if (mark_only) {
    FIA_HIP_TRY(c->mark.reserve((size_t)(U + I), s));
    FIA_HIP_TRY(hipMemsetAsync(c->mark.ptr, 0, (size_t)(U + I), s));
    if (Q > 0) {
      const int64_t gq = (Q + 255) / 256;
      hipLaunchKernelGGL(k_mark_small, dim3((unsigned)(gq < 4096 ? gq : 4096)), dim3(256), 0, s, Q, qu, qi, U, I,
                         c->mark.as<uint8_t>());
      FIA_HIP_TRY(hipGetLastError());
    }
    c->subset = false;
    c->small_subset = false;
    return hipSuccess;
  }
#define X(m, kk, T)                                                     \
  if (c->p.model == m && c->p.k == kk) {                                \
    FIA_HIP_TRY(prepare_impl<T>(c, ps, c->mark.as<uint8_t>()));         \
    c->small_subset = true;                                             \
    return hipSuccess;                                                  \
  }
  FIA_MODEL_CASES(X)
#undef X
  unsupported = true;
  return hipSuccess;
}

hipError_t check_cover_small(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, int32_t* flag,
                             hipStream_t s) {
  if (!c->small_subset || Q <= 0) return hipSuccess;
  const int64_t gq = (Q + 255) / 256;
  hipLaunchKernelGGL(k_check_mark, dim3((unsigned)(gq < 4096 ? gq : 4096)), dim3(256), 0, s, Q, qu, qi, c->p.U, c->p.I,
                     c->mark.as<uint8_t>(), flag);
  return hipGetLastError();
}

hipError_t query_model(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                       int64_t max_chunks, int32_t* rel_idx, double* influence, double* x_out, int K,
                       int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s, bool& unsupported,
                       const double* x_in) {
  unsupported = false;
#define X(m, kk, T)                                                                                        \
  if (c->p.model == m && c->p.k == kk)                                                                     \
    return query_impl<T>(c, Q, qu, qi, offsets, max_chunks, rel_idx, influence, x_out, K, topk_pos, topk_idx, \
                         topk_val, s, x_in);
  FIA_MODEL_CASES(X)
#undef X
  if (big_supported(c->p.model, c->p.k))
    return query_big(c, Q, qu, qi, offsets, max_chunks, rel_idx, influence, x_out, K, topk_pos, topk_idx, topk_val,
                     s, x_in);
  unsupported = true;
  return hipSuccess;
}

}  // namespace fia
