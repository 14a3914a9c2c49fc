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
#include <cstring>

#include "common.h"

namespace fia {
namespace {

// ------------------------------------------------------------------------------------
// model traits
// ------------------------------------------------------------------------------------
template <int K_>
struct MFm {
  static constexpr int K = K_;
  static constexpr int Ds = K + 1;
  static constexpr int D = 2 * Ds;
  static constexpr int SB = 2 * K + 4;          // per-side record: a, xs, bias, xsb, dup_extra, dup_other
  static constexpr int R = 2 + 2 * SB;
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
  static constexpr int SB = 4 * K + 2;          // per-side record: tself, yv, bx, ag, dup_extra, dup_other
  static constexpr int R = 2 + 2 * SB;
  static constexpr bool ncf = true;
  __device__ static bool decayed(int) { return true; }
  // reference theta order [Pm_u, Qm_i, Pg_u, Qg_i]
  __device__ static int ref_index(int a) {
    int side = a >= Ds, j = side ? a - Ds : a;
    return j < K ? side * K + j : 2 * K + side * K + (j - K);
  }
};

__device__ __forceinline__ int tri(int r, int c) { return (r * (r + 1)) / 2 + c; }

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

__device__ __forceinline__ void wave_best(double& a, int& p, double& v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    double oa = __shfl_xor(a, off);
    int op = __shfl_xor(p, off);
    double ov = __shfl_xor(v, off);
    if (better(oa, op, a, p)) { a = oa; p = op; v = ov; }
  }
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

// d1 = ((W2 * (W3m . 1[z2>0])) . 1[z1>0]); returns W3m . relu(z2)
template <int K>
__device__ __forceinline__ double ncf_mlp(const NCFWeights<K>& w, const double (&z1)[K], double (&d1)[K]) {
  constexpr int H = K / 2;
  double z2[H];
#pragma unroll
  for (int d = 0; d < H; ++d) z2[d] = w.b2[d];
#pragma unroll
  for (int c = 0; c < K; ++c) {
    double h = z1[c] > 0.0 ? z1[c] : 0.0;
#pragma unroll
    for (int d = 0; d < H; ++d) z2[d] = fma(w.W2[c * H + d], h, z2[d]);
  }
  double mlp = 0.0, d2[H];
#pragma unroll
  for (int d = 0; d < H; ++d) {
    bool on = z2[d] > 0.0;
    mlp = fma(w.W3[d], on ? z2[d] : 0.0, mlp);
    d2[d] = on ? w.W3[d] : 0.0;
  }
#pragma unroll
  for (int c = 0; c < K; ++c) {
    double t = 0.0;
#pragma unroll
    for (int d = 0; d < H; ++d) t = fma(w.W2[c * H + d], d2[d], t);
    d1[c] = z1[c] > 0.0 ? t : 0.0;
  }
  return mlp;
}

template <int K>
__device__ void load_ncf_weights(NCFWeights<K>& w, const float* W2, const float* b2, const float* W3) {
  constexpr int H = K / 2;
  for (int t = threadIdx.x; t < K * H; t += blockDim.x) w.W2[t] = W2[t];
  for (int t = threadIdx.x; t < H; t += blockDim.x) w.b2[t] = b2[t];
  for (int t = threadIdx.x; t < 3 * H; t += blockDim.x) w.W3[t] = W3[t];
}

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
// Entity Gram: gram[e] = sum over e's rating list of g g^T (packed lower, Ds)
//   MF  g = [emb_other(o) ; 1]
//   NCF g = [W1_self^T-side d1 (k) ; W3g * gmf_other(o) (k)]
// One workgroup per entity; ratings in tiles of TILE, g staged in LDS.
// ------------------------------------------------------------------------------------
template <class M>
struct GramTile {
  static constexpr int TILE = M::ncf ? (M::K <= 16 ? 128 : 64) : 64;
  static constexpr int GS = M::Ds * (M::Ds + 1) / 2;
  static constexpr int MAXE = (GS + kPrepThreads - 1) / kPrepThreads;
  static constexpr int LD = M::Ds + 1;   // padded row
};

template <class M>
__global__ __launch_bounds__(kPrepThreads) void k_gram(
    int side, int64_t n_ent, const int64_t* __restrict__ ptr, const int32_t* __restrict__ other,
    const float* __restrict__ emb_other,      // MF: other side embedding; NCF: other side gmf table
    const double* __restrict__ l1_self, const double* __restrict__ l1_other, const float* __restrict__ W1,
    const float* __restrict__ b1, const float* __restrict__ W2, const float* __restrict__ b2,
    const float* __restrict__ W3, double* __restrict__ gram) {
  using GT = GramTile<M>;
  constexpr int K = M::K, TILE = GT::TILE, LD = GT::LD, GS = GT::GS, MAXE = GT::MAXE;
  __shared__ double g[TILE * LD];
  __shared__ double W1s[M::ncf ? K * K : 1];     // W1 rows of this side, [a][c]
  __shared__ double b1s[M::ncf ? K : 1];
  __shared__ NCFWeights<M::ncf ? K : 2> w;
  const int64_t e = blockIdx.x;
  if (e >= n_ent) return;
  const int tid = threadIdx.x;
  if constexpr (M::ncf) {
    for (int t = tid; t < K * K; t += blockDim.x) W1s[t] = W1[side * K * K + t];
    for (int t = tid; t < K; t += blockDim.x) b1s[t] = b1[t];
    load_ncf_weights<K>(w, W2, b2, W3);
  }
  int er[MAXE], ec[MAXE];
  double acc[MAXE];
#pragma unroll
  for (int m = 0; m < MAXE; ++m) {
    int idx = tid + m * kPrepThreads;
    int r = (int)((sqrtf(8.0f * idx + 1.0f) - 1.0f) * 0.5f);
    while (tri(r + 1, 0) <= idx) ++r;
    while (tri(r, 0) > idx) --r;
    er[m] = r;
    ec[m] = idx - tri(r, 0);
    acc[m] = 0.0;
  }
  const int64_t b = ptr[e], n = ptr[e + 1] - b;
  for (int64_t t0 = 0; t0 < n; t0 += TILE) {
    const int rows = (int)((n - t0) < TILE ? (n - t0) : TILE);
    __syncthreads();
    for (int t = tid; t < rows; t += blockDim.x) {
      const int32_t o = other[b + t0 + t];
      double* gr = g + t * LD;
      if constexpr (!M::ncf) {
        double row[K];
        load_row_f32<K>(emb_other + (int64_t)o * K, row);
#pragma unroll
        for (int c = 0; c < K; ++c) gr[c] = row[c];
        gr[K] = 1.0;
      } else {
        constexpr int H = K / 2;
        double z1[K], d1[K];
#pragma unroll
        for (int c = 0; c < K; ++c) z1[c] = l1_self[e * K + c] + l1_other[(int64_t)o * K + c] + b1s[c];
        (void)ncf_mlp<K>(w, z1, d1);
#pragma unroll
        for (int a = 0; a < K; ++a) {
          double s = 0.0;
#pragma unroll
          for (int c = 0; c < K; ++c) s = fma(W1s[a * K + c], d1[c], s);
          gr[a] = s;
        }
        double row[K];
        load_row_f32<K>(emb_other + (int64_t)o * K, row);
#pragma unroll
        for (int a = 0; a < K; ++a) gr[K + a] = w.W3[H + a] * row[a];
      }
    }
    __syncthreads();
#pragma unroll
    for (int m = 0; m < MAXE; ++m) {
      if (tid + m * kPrepThreads < GS) {
        const double* pr = g + er[m];
        const double* pc = g + ec[m];
        double s = acc[m];
        for (int t = 0; t < rows; ++t) s = fma(pr[t * LD], pc[t * LD], s);
        acc[m] = s;
      }
    }
  }
  double* out = gram + e * GS;
#pragma unroll
  for (int m = 0; m < MAXE; ++m) {
    int idx = tid + m * kPrepThreads;
    if (idx < GS) out[idx] = acc[m];
  }
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
};

template <class M>
__global__ __launch_bounds__(kSolveThreads) void k_solve(QueryArgs A, int64_t Q, double* __restrict__ rec,
                                                         double* __restrict__ x_out) {
  constexpr int K = M::K, Ds = M::Ds, D = M::D, GS = Ds * (Ds + 1) / 2;
  __shared__ double H[D * (D + 1) / 2];
  __shared__ double v[D], g[D], th[D], dd[D], ww[D];
  __shared__ double sh[4 * K + 8];
  const int64_t q = blockIdx.x;
  if (q >= Q) return;
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
    return;
  }
  const double s2n = 2.0 / (double)n;

  // ---- theta_t and v = d r(u,i)/d theta_t (gnn:155, mf:194,201 / ncf:222,229) ----
  double rhat_ui = 0.0;
  if constexpr (!M::ncf) {
    const float* P = A.t[0];
    const float* Qt = A.t[1];
    for (int a = lane; a < K; a += kSolveThreads) {
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
    for (int a = lane; a < K; a += kSolveThreads) part += th[a] * th[Ds + a];
    rhat_ui = wave_sum(part) + th[K] + th[Ds + K] + (double)A.t[4][0];
  } else {
    constexpr int H2 = K / 2;
    const float* Pm = A.t[0];
    const float* Qm = A.t[1];
    const float* Pg = A.t[2];
    const float* Qg = A.t[3];
    const float* W1 = A.t[4];
    const float* b1 = A.t[5];
    const float* W2 = A.t[6];
    const float* b2 = A.t[7];
    const float* W3 = A.t[8];
    double* z1 = sh;            // K
    double* d2 = sh + K;        // K/2
    double* d1 = sh + 2 * K;    // K
    for (int a = lane; a < K; a += kSolveThreads) {
      th[a] = Pm[(int64_t)u * K + a];
      th[K + a] = Pg[(int64_t)u * K + a];
      th[Ds + a] = Qm[(int64_t)i * K + a];
      th[Ds + K + a] = Qg[(int64_t)i * K + a];
      z1[a] = A.l1[0][(int64_t)u * K + a] + A.l1[1][(int64_t)i * K + a] + (double)b1[a];
    }
    __syncthreads();
    double mlp_part = 0.0;
    for (int dd2 = lane; dd2 < H2; dd2 += kSolveThreads) {
      double z2 = b2[dd2];
      for (int c = 0; c < K; ++c) z2 = fma((double)W2[c * H2 + dd2], z1[c] > 0.0 ? z1[c] : 0.0, z2);
      const bool on = z2 > 0.0;
      d2[dd2] = on ? (double)W3[dd2] : 0.0;
      mlp_part += on ? (double)W3[dd2] * z2 : 0.0;
    }
    double gmf_part = 0.0;
    for (int a = lane; a < K; a += kSolveThreads) gmf_part += (double)W3[H2 + a] * th[K + a] * th[Ds + K + a];
    rhat_ui = wave_sum(mlp_part + gmf_part) + (double)A.t[9][0];
    __syncthreads();
    for (int c = lane; c < K; c += kSolveThreads) {
      double t = 0.0;
      for (int dd2 = 0; dd2 < H2; ++dd2) t = fma((double)W2[c * H2 + dd2], d2[dd2], t);
      d1[c] = z1[c] > 0.0 ? t : 0.0;
    }
    __syncthreads();
    for (int a = lane; a < 2 * K; a += kSolveThreads) {
      // rows a < K: W1[:k] (Pm part, user block); rows a >= K: W1[k:] (Qm part, item block)
      double s = 0.0;
      for (int c = 0; c < K; ++c) s = fma((double)W1[a * K + c], d1[c], s);
      if (a < K) g[a] = s; else g[Ds + (a - K)] = s;
    }
    for (int a = lane; a < K; a += kSolveThreads) {
      g[K + a] = (double)W3[H2 + a] * th[Ds + K + a];        // d r/d Pg_u = W3g * Qg_i
      g[Ds + K + a] = (double)W3[H2 + a] * th[K + a];        // d r/d Qg_i = W3g * Pg_u
    }
  }
  __syncthreads();

  // ---- the (u,i) pair among the train rows: scan the shorter list ----
  double cdup = 0.0, rsum = 0.0;
  {
    const int sd = du <= di ? 0 : 1;
    const int64_t lb = sd == 0 ? ub : ib, ln = sd == 0 ? du : di;
    const int32_t want = sd == 0 ? i : u;
    const int32_t* oth = A.other[sd] + lb;
    const float* rt = A.rating[sd] + lb;
    for (int64_t p = lane; p < ln; p += kSolveThreads)
      if (oth[p] == want) { cdup += 1.0; rsum += (double)rt[p]; }
    cdup = wave_sum(cdup);
    rsum = wave_sum(rsum);
  }
  const bool coupled = cdup > 0.0;
  const double esum = cdup * rhat_ui - rsum;

  // ---- assemble H (packed lower, D x D) ----
  const double* Gu = A.gram[0] + (int64_t)u * GS;
  const double* Gi = A.gram[1] + (int64_t)i * GS;
  for (int t = lane; t < D * (D + 1) / 2; t += kSolveThreads) {
    int r = (int)((sqrt(8.0 * t + 1.0) - 1.0) * 0.5);
    while (tri(r + 1, 0) <= t) ++r;
    while (tri(r, 0) > t) --r;
    const int c = t - tri(r, 0);
    double h = 0.0;
    if (r < Ds) {
      h = s2n * (Gu[tri(r, c)] + cdup * g[r] * g[c]);
    } else if (c >= Ds) {
      const int rr = r - Ds, cc = c - Ds;
      h = s2n * (Gi[tri(rr, cc)] + cdup * g[r] * g[c]);
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

  // ---- outputs ----
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
  if (lane == 0) {
    R[0] = 1.0 / (double)n;
    R[1] = cq;
  }
  double* S0 = R + 2;
  double* S1 = R + 2 + M::SB;
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
      S0[2 * K + 2] = xg_item;    S1[2 * K + 2] = xg_user;
      S0[2 * K + 3] = (double)i;  S1[2 * K + 3] = (double)u;
    }
  } else {
    constexpr int H2 = K / 2;
    const float* W1 = A.t[4];
    const float* b1 = A.t[5];
    const float* W3 = A.t[8];
    for (int c = lane; c < K; c += kSolveThreads) {
      S0[c] = A.l1[0][(int64_t)u * K + c] + (double)b1[c];
      S1[c] = A.l1[1][(int64_t)i * K + c] + (double)b1[c];
      double y0 = 0.0, y1 = 0.0;
      for (int a = 0; a < K; ++a) {
        y0 = fma(v[a], (double)W1[a * K + c], y0);
        y1 = fma(v[Ds + a], (double)W1[(K + a) * K + c], y1);
      }
      S0[K + c] = y0;
      S1[K + c] = y1;
      const double w3g = (double)W3[H2 + c];
      S0[2 * K + c] = w3g * v[K + c];
      S1[2 * K + c] = w3g * v[Ds + K + c];
      S0[3 * K + c] = w3g * th[K + c];
      S1[3 * K + c] = w3g * th[Ds + K + c];
    }
    if (lane == 0) {
      S0[4 * K] = xg_item;   S1[4 * K] = xg_user;
      S0[4 * K + 1] = (double)i;  S1[4 * K + 1] = (double)u;
    }
  }
}

// ------------------------------------------------------------------------------------
// Scoring: one workgroup per chunk of <= kChunk related ratings of one query.
// influence = (2 e s + c_q) / n with s = x . g_j (mf:240-246)
// ------------------------------------------------------------------------------------
template <class M>
__global__ __launch_bounds__(kScoreThreads) void k_score(
    QueryArgs A, int64_t Q, const int64_t* __restrict__ offsets, const int64_t* __restrict__ coff,
    const int32_t* __restrict__ cquery, const int32_t* __restrict__ cstart, const double* __restrict__ rec,
    int64_t* __restrict__ rel_idx, double* __restrict__ influence, int K_top, int32_t* __restrict__ cand_pos,
    double* __restrict__ cand_val) {
  constexpr int K = M::K;
  __shared__ double sr[M::R];
  __shared__ NCFWeights<M::ncf ? K : 2> w;
  __shared__ double s_a[kScoreThreads / 64], s_v[kScoreThreads / 64];
  __shared__ int s_p[kScoreThreads / 64];
  const int64_t nchunks = coff[Q];
  const int tid = threadIdx.x;
  if constexpr (M::ncf) {
    load_ncf_weights<K>(w, A.t[6], A.t[7], A.t[8]);
  }
  for (int64_t ch = blockIdx.x; ch < nchunks; ch += gridDim.x) {
    const int32_t q = cquery[ch];
    const int32_t start = cstart[ch];
    const int32_t u = A.qu[q], i = A.qi[q];
    const int64_t ub = A.ptr[0][u], du = A.ptr[0][u + 1] - ub;
    const int64_t ib = A.ptr[1][i];
    const int64_t base = offsets[q];
    const int64_t n = offsets[q + 1] - base;
    __syncthreads();
    for (int t = tid; t < M::R; t += kScoreThreads) sr[t] = rec[(int64_t)q * M::R + t];
    __syncthreads();
    const double inv_n = sr[0], cq = sr[1];
    double ca[kScoreRows], cv[kScoreRows];
    int cp[kScoreRows];
#pragma unroll
    for (int rr = 0; rr < kScoreRows; ++rr) {
      const int64_t p = (int64_t)start + rr * kScoreThreads + tid;
      cp[rr] = -1;
      ca[rr] = -2.0;
      cv[rr] = 0.0;
      if (p >= n) continue;
      const int sd = p < du ? 0 : 1;
      const int64_t li = sd == 0 ? ub + p : ib + (p - du);
      const int32_t o = A.other[sd][li];
      const double y = (double)A.rating[sd][li];
      const double* S = sr + 2 + sd * M::SB;
      double infl;
      if constexpr (!M::ncf) {
        // other-side embedding and bias: side 0 (user rows) -> item tables, side 1 -> user tables
        const float* T = sd == 0 ? A.t[1] : A.t[0];
        const float* bt = sd == 0 ? A.t[3] : A.t[2];
        double row_e[K];
        load_row_f32<K>(T + (int64_t)o * K, row_e);
        double dot_a = 0.0, dot_x = 0.0;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          dot_a = fma(S[c], row_e[c], dot_a);
          dot_x = fma(S[K + c], row_e[c], dot_x);
        }
        const double e = dot_a + S[2 * K] + (double)bt[o] - y;
        double s = dot_x + S[2 * K + 1];
        if ((double)o == S[2 * K + 3]) s += S[2 * K + 2];
        infl = (2.0 * e * s + cq) * inv_n;
      } else {
        constexpr int H2 = K / 2;
        const double* L1o = A.l1[sd == 0 ? 1 : 0] + (int64_t)o * K;
        const float* G = (sd == 0 ? A.t[3] : A.t[2]) + (int64_t)o * K;   // other side gmf row
        double z1[K], d1[K], grow[K];
#pragma unroll
        for (int c = 0; c < K; ++c) z1[c] = S[c] + L1o[c];
        const double mlp = ncf_mlp<K>(w, z1, d1);
        load_row_f32<K>(G, grow);
        double gmf = 0.0, s = 0.0;
#pragma unroll
        for (int c = 0; c < K; ++c) {
          s = fma(S[K + c], d1[c], s);
          s = fma(S[2 * K + c], grow[c], s);
          gmf = fma(S[3 * K + c], grow[c], gmf);
        }
        (void)H2;
        const double e = mlp + gmf + (double)A.t[9][0] - y;
        if ((double)o == S[4 * K + 1]) s += S[4 * K];
        infl = (2.0 * e * s + cq) * inv_n;
      }
      if (influence) influence[base + p] = infl;
      if (rel_idx) rel_idx[base + p] = A.row[sd][li];
      cp[rr] = (int)p;
      ca[rr] = topk_key(infl);
      cv[rr] = infl;
    }
    if (K_top > 0)
      block_topk<kScoreRows, kScoreThreads>(ca, cp, cv, K_top, cand_pos + ch * K_top, cand_val + ch * K_top, s_a, s_p,
                                            s_v);
  }
}

// Merge the chunk candidates of every query (one wave per query).
__global__ __launch_bounds__(64) void k_topk_merge(const int32_t* __restrict__ qu, const int32_t* __restrict__ qi,
                                                   int64_t Q, const int64_t* __restrict__ coff, int K,
                                                   const int32_t* __restrict__ cand_pos,
                                                   const double* __restrict__ cand_val,
                                                   const int64_t* __restrict__ uptr, const int32_t* __restrict__ urow,
                                                   const int64_t* __restrict__ iptr, const int32_t* __restrict__ irow,
                                                   int64_t U, int64_t I, int64_t* __restrict__ topk_pos,
                                                   int64_t* __restrict__ topk_idx, double* __restrict__ topk_val) {
  const int64_t q = blockIdx.x;
  if (q >= Q) return;
  const int lane = threadIdx.x;
  const int64_t cb = coff[q] * K, ce = coff[q + 1] * K;
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

// ------------------------------------------------------------------------------------
// host-side dispatch
// ------------------------------------------------------------------------------------
QueryArgs make_args(fia_ctx* c, const int32_t* qu, const int32_t* qi) {
  QueryArgs A;
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
  return A;
}

template <class M>
hipError_t prepare_impl(fia_ctx* c, hipStream_t s) {
  constexpr int Ds = M::Ds, GS = Ds * (Ds + 1) / 2, K = M::K;
  const int64_t n_ent[2] = {c->p.U, c->p.I};
  for (int sd = 0; sd < 2; ++sd) FIA_HIP_TRY(c->gram[sd].reserve(sizeof(double) * (size_t)(n_ent[sd] * GS + 1)));
  if constexpr (M::ncf) {
    for (int sd = 0; sd < 2; ++sd) {
      FIA_HIP_TRY(c->l1[sd].reserve(sizeof(double) * (size_t)(n_ent[sd] * K + 1)));
      const int64_t tot = n_ent[sd] * K;
      if (tot > 0) {
        hipLaunchKernelGGL(k_ncf_l1<K>, dim3((unsigned)((tot + 255) / 256)), dim3(256), 0, s, c->p.t[sd],
                           c->p.t[4], sd * K, n_ent[sd], c->l1[sd].as<double>());
        FIA_HIP_TRY(hipGetLastError());
      }
    }
  }
  for (int sd = 0; sd < 2; ++sd) {
    if (n_ent[sd] == 0) continue;
    const float* emb_other;
    if constexpr (M::ncf) emb_other = c->p.t[sd == 0 ? 3 : 2];   // gmf table of the other side
    else emb_other = c->p.t[sd == 0 ? 1 : 0];
    hipLaunchKernelGGL(k_gram<M>, dim3((unsigned)n_ent[sd]), dim3(kPrepThreads), 0, s, sd, n_ent[sd],
                       c->idx.side[sd].ptr.as<int64_t>(), c->idx.side[sd].other.as<int32_t>(), emb_other,
                       c->l1[sd].as<double>(), c->l1[1 - sd].as<double>(), c->p.t[4], c->p.t[5], c->p.t[6],
                       c->p.t[7], c->p.t[8], c->gram[sd].as<double>());
    FIA_HIP_TRY(hipGetLastError());
  }
  return hipSuccess;
}

template <class M>
hipError_t query_impl(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                      int64_t max_chunks, int64_t* rel_idx, double* influence, double* x_out, int K,
                      int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s) {
  FIA_HIP_TRY(c->rec.reserve(sizeof(double) * (size_t)(Q * M::R + 1)));
  if (K > 0) {
    FIA_HIP_TRY(c->cand_pos.reserve(sizeof(int32_t) * (size_t)((max_chunks + 1) * K)));
    FIA_HIP_TRY(c->cand_val.reserve(sizeof(double) * (size_t)((max_chunks + 1) * K)));
  }
  QueryArgs A = make_args(c, qu, qi);
  phase_begin(c, 4, s);
  FIA_HIP_TRY(build_chunks(c, Q, offsets, max_chunks, s));
  phase_end(c, 4, s);
  phase_begin(c, 1, s);
  hipLaunchKernelGGL(k_solve<M>, dim3((unsigned)Q), dim3(kSolveThreads), 0, s, A, Q, c->rec.as<double>(), x_out);
  FIA_HIP_TRY(hipGetLastError());
  phase_end(c, 1, s);
  int64_t grid = max_chunks < 1 ? 1 : max_chunks;
  if (grid > 16384) grid = 16384;
  phase_begin(c, 2, s);
  hipLaunchKernelGGL(k_score<M>, dim3((unsigned)grid), dim3(kScoreThreads), 0, s, A, Q, offsets,
                     c->coff.as<int64_t>(), c->cquery.as<int32_t>(), c->cstart.as<int32_t>(), c->rec.as<double>(),
                     rel_idx, influence, K, c->cand_pos.as<int32_t>(), c->cand_val.as<double>());
  FIA_HIP_TRY(hipGetLastError());
  phase_end(c, 2, s);
  if (K > 0 && Q > 0) {
    phase_begin(c, 3, s);
    hipLaunchKernelGGL(k_topk_merge, dim3((unsigned)Q), dim3(64), 0, s, qu, qi, Q, c->coff.as<int64_t>(), K,
                       c->cand_pos.as<int32_t>(), c->cand_val.as<double>(), c->idx.side[0].ptr.as<int64_t>(),
                       c->idx.side[0].row.as<int32_t>(), c->idx.side[1].ptr.as<int64_t>(),
                       c->idx.side[1].row.as<int32_t>(), c->p.U, c->p.I, topk_pos, topk_idx, topk_val);
    FIA_HIP_TRY(hipGetLastError());
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
  return false;
}

int model_num_params(int model, int k) {
  if (model == FIA_MODEL_MF) return 2 * k + 2;
  if (model == FIA_MODEL_NCF) return 4 * k;
  return 0;
}

hipError_t prepare_model(fia_ctx* c, hipStream_t s, bool& unsupported) {
  unsupported = false;
#define X(m, kk, T) if (c->p.model == m && c->p.k == kk) return prepare_impl<T>(c, s);
  FIA_MODEL_CASES(X)
#undef X
  unsupported = true;
  return hipSuccess;
}

hipError_t query_model(fia_ctx* c, int64_t Q, const int32_t* qu, const int32_t* qi, const int64_t* offsets,
                       int64_t max_chunks, int64_t* rel_idx, double* influence, double* x_out, int K,
                       int64_t* topk_pos, int64_t* topk_idx, double* topk_val, hipStream_t s, bool& unsupported) {
  unsupported = false;
#define X(m, kk, T)                                                                                        \
  if (c->p.model == m && c->p.k == kk)                                                                     \
    return query_impl<T>(c, Q, qu, qi, offsets, max_chunks, rel_idx, influence, x_out, K, topk_pos, topk_idx, \
                         topk_val, s);
  FIA_MODEL_CASES(X)
#undef X
  unsupported = true;
  return hipSuccess;
}

}  // namespace fia
