// CPU-side runtime for the data pipeline (built with g++ -O3 -fopenmp into
// libmda_host.so, loaded through ctypes by ops/_ext.py).
//
//  * mdah_crd_sample  -- CRD contrastive index sampling for a whole batch:
//    positive (exact: the sample itself; relax: a random same-class sample)
//    + K negatives drawn uniformly from the other classes, without
//    replacement (Robert Floyd's algorithm, O(K) per sample) or with
//    replacement, exactly the distributions of the reference datasets
//    (dataset/cifar100.py:83-113, tiny_imagenet.py, imagenet.py).  OpenMP
//    over the batch; a counter-based per-(seed, sample) RNG makes the result
//    independent of the thread count.
//  * mdah_alias_build -- Walker alias table (reference AliasMethod,
//    distillers/CRD.py:223-281) for non-uniform negative distributions.
#include <stdint.h>
#include <string.h>

#include <unordered_set>
#include <vector>

#define MDA_HOST_API extern "C" __attribute__((visibility("default")))

namespace {

struct SplitMix64 {
  uint64_t s;
  explicit SplitMix64(uint64_t seed) : s(seed) {}
  uint64_t next() {
    uint64_t z = (s += 0x9e3779b97f4a7c15ULL);
    z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
    z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
    return z ^ (z >> 31);
  }
  // uniform integer in [0, n)
  uint64_t below(uint64_t n) {
    // Lemire's nearly-divisionless method
    uint64_t x = next();
    __uint128_t m = (__uint128_t)x * n;
    uint64_t l = (uint64_t)m;
    if (l < n) {
      uint64_t t = (0 - n) % n;
      while (l < t) {
        x = next();
        m = (__uint128_t)x * n;
        l = (uint64_t)m;
      }
    }
    return (uint64_t)(m >> 64);
  }
};

// r-th element (0-based) of the samples NOT in class c, given samples sorted by class
inline int64_t nth_negative(const int64_t* sorted, int64_t start_c, int64_t count_c, int64_t r) {
  return r < start_c ? sorted[r] : sorted[r + count_c];
}

}  // namespace

// cls_sorted[N]: sample indices grouped by class; cls_start/cls_count[C];
// targets[B], index[B]; out[B, K+1].  Returns 0 on success.
MDA_HOST_API int mdah_crd_sample(const int64_t* cls_sorted, const int64_t* cls_start,
                                 const int64_t* cls_count, const int64_t* targets,
                                 const int64_t* index, int64_t* out, int64_t B, int64_t K,
                                 int64_t N, int64_t flags, int64_t seed) {
  const bool replace = flags & 1;
  const bool relax = flags & 2;
#pragma omp parallel for schedule(dynamic, 4)
  for (int64_t b = 0; b < B; ++b) {
    SplitMix64 rng((uint64_t)seed * 0x100000001b3ULL + (uint64_t)index[b] * 0x9e37ULL + b);
    const int64_t c = targets[b];
    const int64_t st = cls_start[c], cnt = cls_count[c];
    const int64_t nneg = N - cnt;
    int64_t* o = out + b * (K + 1);
    o[0] = relax ? cls_sorted[st + (int64_t)rng.below((uint64_t)cnt)] : index[b];
    if (replace || K > nneg) {
      for (int64_t k = 0; k < K; ++k) o[1 + k] = nth_negative(cls_sorted, st, cnt, (int64_t)rng.below((uint64_t)nneg));
    } else {
      // Floyd: K distinct ranks from [0, nneg)
      std::unordered_set<int64_t> seen;
      seen.reserve((size_t)K * 2);
      int64_t k = 0;
      for (int64_t j = nneg - K; j < nneg; ++j) {
        int64_t t = (int64_t)rng.below((uint64_t)(j + 1));
        int64_t pick = seen.insert(t).second ? t : (seen.insert(j), j);
        o[1 + k++] = nth_negative(cls_sorted, st, cnt, pick);
      }
    }
  }
  return 0;
}

// probs[K] (normalised or not) -> prob_out[K] (float), alias_out[K]
MDA_HOST_API int mdah_alias_build(const double* probs, float* prob_out, int64_t* alias_out,
                                  int64_t K) {
  double total = 0;
  for (int64_t i = 0; i < K; ++i) total += probs[i];
  std::vector<double> q(K);
  std::vector<int64_t> small, large;
  for (int64_t i = 0; i < K; ++i) {
    q[i] = K * probs[i] / total;
    alias_out[i] = 0;
    (q[i] < 1.0 ? small : large).push_back(i);
  }
  while (!small.empty() && !large.empty()) {
    int64_t s = small.back(); small.pop_back();
    int64_t l = large.back(); large.pop_back();
    alias_out[s] = l;
    q[l] = (q[l] - 1.0) + q[s];
    (q[l] < 1.0 ? small : large).push_back(l);
  }
  for (int64_t i : small) q[i] = 1.0;
  for (int64_t i : large) q[i] = 1.0;
  for (int64_t i = 0; i < K; ++i) prob_out[i] = (float)q[i];
  return 0;
}
