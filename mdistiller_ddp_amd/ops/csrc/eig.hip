// Batched symmetric eigendecomposition of small Gram matrices, for KDSVD
// (reference distillers/KDSVD.py:8-35 takes torch.svd of each sample's
// (C*H) x W feature view and uses the right singular vectors V and the
// singular values).  V and sigma^2 are the eigenvectors / eigenvalues of the
// W x W Gram G = X^T X, so the SVD reduces to a tiny eigenproblem per sample.
//
// rocSOLVER's batched SVD / syevd check their info word on the host, which
// breaks hipGraph capture; this kernel has no host interaction:
//
//   * one workgroup per matrix (n <= 63), the matrix (fp64) and the
//     accumulated rotations (fp32) live in LDS (< 64 KB); odd n gets a zero row / column (its
//     rotations are exactly the identity, so it never mixes and is dropped);
//   * parallel cyclic Jacobi: each step applies n/2 disjoint rotations
//     (round-robin tournament pairing, n-1 steps per sweep), a fixed number of
//     sweeps at most (quadratic convergence: 8 sweeps reach fp64 round-off for
//     n <= 64), stopping early once the off-diagonal mass is negligible;
//   * eigenvalues sorted descending (rank by comparison, ties by index),
//     each eigenvector's sign fixed so its largest-magnitude component is
//     positive (LAPACK's sign is arbitrary; this one is deterministic).
//
// Output: vals [B][n] (descending), vecs [B][n][n] row-major with the
// eigenvectors as COLUMNS (V[:, j] pairs with vals[j]), fp32.
#include <algorithm>
#include <cstdlib>

#include "common.h"

namespace {

constexpr int EIG_NMAX = 64;
constexpr int EIG_MAXE = 8;

// One batch of matrices per table entry (blockIdx.y): B matrices of size n0,
// the input summed over `parts` partial Grams (part stride pstride floats --
// csrc/kdsvd.hip's split-K Gram), results at vals / vecs.  Entries of
// different sizes run side by side in ONE launch (KDSVD's stages: the small
// matrices finish under the largest one's sweeps instead of after them).
struct EigEntry {
  const float* g; float* vals; float* vecs;
  int64_t pstride;
  int B, n0, parts;
};
struct EigTable { EigEntry e[EIG_MAXE]; };

__global__ void __launch_bounds__(256) sym_eig_kernel(EigTable tab, int sweeps) {
  __shared__ double A[EIG_NMAX][EIG_NMAX + 1];
  __shared__ float V[EIG_NMAX][EIG_NMAX + 1];  // rotations accumulated in fp32
  __shared__ double cs[EIG_NMAX / 2][2];
  __shared__ int pp[EIG_NMAX / 2], qq[EIG_NMAX / 2];  // this step's pairs
  __shared__ double lam[EIG_NMAX];
  __shared__ int order[EIG_NMAX];
  __shared__ double red[2][8];
  const EigEntry& en = tab.e[blockIdx.y];
  const int b = blockIdx.x, tid = threadIdx.x, nt = blockDim.x;
  if (b >= en.B) return;  // uniform per block: before any barrier
  const int n0 = en.n0;
  float* __restrict__ vals = en.vals;
  float* __restrict__ vecs = en.vecs;
  const float* gb = en.g + (int64_t)b * n0 * n0;
  const int n = n0 + (n0 & 1);
  // e -> (e / n, e % n) by shift / mask when n is a power of two (the KDSVD
  // sizes 8 / 16 / 32): the row / column phases run it every Jacobi step
  const int lgn = (n & (n - 1)) == 0 ? __builtin_ctz(n) : -1;
  auto divn = [&](int e, int& a, int& b) {
    if (lgn >= 0) { a = e >> lgn; b = e & (n - 1); }
    else { a = e / n; b = e - (e / n) * n; }
  };
  for (int e = tid; e < n * n; e += nt) {
    const int i = e / n, j = e % n;
    // symmetrise (G is symmetric up to the GEMM's rounding), summing the parts
    double a = 0.0;
    if (i < n0 && j < n0)
      for (int q = 0; q < en.parts; ++q)
        a += (double)gb[q * en.pstride + i * n0 + j] + (double)gb[q * en.pstride + j * n0 + i];
    A[i][j] = 0.5 * a;
    V[i][j] = i == j ? 1.f : 0.f;
  }
  const int m = n - 1, half = n / 2;
  __syncthreads();
  for (int sw = 0; sw < sweeps; ++sw) {
    // converged (off-diagonal mass below 1e-22 of the total): every further
    // rotation would be the identity to fp32 output precision
    {
      double off = 0.0, tot = 0.0;
      for (int e = tid; e < n * n; e += nt) {
        int i, j;
        divn(e, i, j);
        const double a2 = A[i][j] * A[i][j];
        tot += a2;
        off += i == j ? 0.0 : a2;
      }
      for (int o = 32; o > 0; o >>= 1) {
        off += __shfl_xor(off, o);
        tot += __shfl_xor(tot, o);
      }
      if ((tid & 63) == 0) { red[0][tid >> 6] = off; red[1][tid >> 6] = tot; }
      __syncthreads();
      off = tot = 0.0;
      for (int w = 0; w < (nt >> 6); ++w) { off += red[0][w]; tot += red[1][w]; }
      __syncthreads();
      if (off <= 1e-22 * tot) break;  // uniform across the block
    }
    for (int r = 0; r < m; ++r) {
      // round-robin pairing: (m, r) and ((r+k) % m, (r-k+m) % m), k = 1..half-1
      if (tid < half) {
        int p, q;
        if (tid == 0) {
          p = r; q = m;
        } else {
          p = (r + tid) % m; q = (r - tid + m) % m;
        }
        if (p > q) { const int t = p; p = q; q = t; }
        const double apq = A[p][q];
        double c = 1.0, s = 0.0;
        if (apq != 0.0) {
          const double theta = (A[q][q] - A[p][p]) / (2.0 * apq);
          const double t = (theta >= 0.0 ? 1.0 : -1.0) / (fabs(theta) + sqrt(theta * theta + 1.0));
          c = 1.0 / sqrt(t * t + 1.0);
          s = t * c;
        }
        cs[tid][0] = c; cs[tid][1] = s;
        pp[tid] = p; qq[tid] = q;
      }
      __syncthreads();
      // rows, in place per pair: A <- J^T A
      for (int e = tid; e < half * n; e += nt) {
        int k, j;
        divn(e, k, j);
        const int p = pp[k], q = qq[k];
        const double c = cs[k][0], s = cs[k][1], ap = A[p][j], aq = A[q][j];
        A[p][j] = c * ap - s * aq;
        A[q][j] = s * ap + c * aq;
      }
      __syncthreads();
      // columns, in place per pair: A <- A J, V <- V J
      for (int e = tid; e < half * n; e += nt) {
        int k, i;
        divn(e, k, i);
        const int p = pp[k], q = qq[k];
        const double c = cs[k][0], s = cs[k][1], ap = A[i][p], aq = A[i][q];
        A[i][p] = c * ap - s * aq;
        A[i][q] = s * ap + c * aq;
        const float cf = (float)c, sf = (float)s, vp = V[i][p], vq = V[i][q];
        V[i][p] = cf * vp - sf * vq;
        V[i][q] = sf * vp + cf * vq;
      }
      __syncthreads();
    }
  }
  for (int i = tid; i < n0; i += nt) lam[i] = A[i][i];
  __syncthreads();
  for (int i = tid; i < n0; i += nt) {
    int rank = 0;
    for (int j = 0; j < n0; ++j) rank += (lam[j] > lam[i]) || (lam[j] == lam[i] && j < i);
    order[rank] = i;
  }
  __syncthreads();
  float* vb = vecs + (int64_t)b * n0 * n0;
  for (int jj = tid; jj < n0; jj += nt) {
    const int j = order[jj];
    vals[(int64_t)b * n0 + jj] = (float)lam[j];
    int im = 0;
    double best = -1.0;
    for (int i = 0; i < n0; ++i) {
      const double a = fabsf(V[i][j]);
      if (a > best) { best = a; im = i; }
    }
    const double sg = V[im][j] < 0.0 ? -1.0 : 1.0;
    for (int i = 0; i < n0; ++i) vb[i * n0 + jj] = (float)(sg * V[i][j]);
  }
}

}  // namespace

static int eig_threads() {
  // block size (64 / 128 / 256; MDA_EIG_THREADS): the Jacobi steps are
  // latency bound, fewer waves make each step's barriers cheaper
  static const int threads = [] {
    const char* e = getenv("MDA_EIG_THREADS");
    const int t = e ? atoi(e) : 256;
    return (t == 64 || t == 128) ? t : 256;
  }();
  return threads;
}

// g: [B][n][n] fp32 symmetric (n <= 63); vals [B][n], vecs [B][n][n] fp32 (see above).
MDA_API int mda_sym_eig(const float* g, int64_t B, int64_t n, int64_t sweeps, float* vals,
                        float* vecs, hipStream_t st) {
  if (B <= 0 || B > 65535 || n < 2 || n >= EIG_NMAX || sweeps < 1 || sweeps > 64)
    return (int)hipErrorInvalidValue;
  EigTable tab{};
  tab.e[0] = EigEntry{g, vals, vecs, 0, (int)B, (int)n, 1};
  hipLaunchKernelGGL(sym_eig_kernel, dim3((unsigned)B), dim3(eig_threads()), 0, st, tab, (int)sweeps);
  return (int)hipGetLastError();
}

// Several batches in one launch.  table: int64 [E][7] rows
// (g, vals, vecs, pstride, B, n, parts); E <= 8.
MDA_API int mda_sym_eig_multi(const int64_t* table, int64_t E, int64_t sweeps, hipStream_t st) {
  if (E < 1 || E > EIG_MAXE || sweeps < 1 || sweeps > 64) return (int)hipErrorInvalidValue;
  EigTable tab{};
  int bmax = 0;
  for (int e = 0; e < E; ++e) {
    const int64_t* r = table + 7 * e;
    if (r[4] <= 0 || r[4] > 65535 || r[5] < 2 || r[5] >= EIG_NMAX || r[6] < 1 || r[6] > 64)
      return (int)hipErrorInvalidValue;
    tab.e[e] = EigEntry{(const float*)r[0], (float*)r[1], (float*)r[2], r[3], (int)r[4], (int)r[5],
                        (int)r[6]};
    bmax = std::max(bmax, (int)r[4]);
  }
  hipLaunchKernelGGL(sym_eig_kernel, dim3((unsigned)bmax, (unsigned)E), dim3(eig_threads()), 0, st,
                     tab, (int)sweeps);
  return (int)hipGetLastError();
}
