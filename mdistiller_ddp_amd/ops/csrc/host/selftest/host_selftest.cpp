// Self-test driver for the CPU runtime (csrc/host/*.cpp), built by
// ops/build.py::build_host_sanitized() with AddressSanitizer + UBSan
// (sanitizer coverage of the native host code).  Exercises every
// exported entry point over several shapes and checks the invariants the
// Python side relies on; any out-of-bounds access, leak or UB aborts with a
// sanitizer report.  Exit code 0 = all checks passed.
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

#include <algorithm>
#include <set>
#include <vector>

extern "C" int mdah_crd_sample(const int64_t* cls_sorted, const int64_t* cls_start,
                               const int64_t* cls_count, const int64_t* targets,
                               const int64_t* index, int64_t* out, int64_t B, int64_t K,
                               int64_t N, int64_t flags, int64_t seed);
extern "C" int mdah_alias_build(const double* probs, float* prob_out, int64_t* alias_out,
                                int64_t K);

static int g_fail = 0;
#define CHECK(c, ...)                         \
  do {                                        \
    if (!(c)) {                               \
      fprintf(stderr, "FAIL %s:%d ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);           \
      fprintf(stderr, "\n");                  \
      ++g_fail;                               \
    }                                         \
  } while (0)

static void crd_case(int64_t N, int64_t C, int64_t B, int64_t K, int64_t flags) {
  std::vector<int64_t> label(N), sorted(N), start(C), count(C, 0);
  for (int64_t i = 0; i < N; ++i) label[i] = (i * 7 + 3) % C;
  for (int64_t i = 0; i < N; ++i) ++count[label[i]];
  for (int64_t c = 0, s = 0; c < C; ++c) { start[c] = s; s += count[c]; }
  std::vector<int64_t> fill(start);
  for (int64_t i = 0; i < N; ++i) sorted[fill[label[i]]++] = i;
  std::vector<int64_t> idx(B), tgt(B), out(B * (K + 1), -1);
  for (int64_t b = 0; b < B; ++b) { idx[b] = (b * 31) % N; tgt[b] = label[idx[b]]; }
  int rc = mdah_crd_sample(sorted.data(), start.data(), count.data(), tgt.data(), idx.data(),
                           out.data(), B, K, N, flags, 1234);
  CHECK(rc == 0, "rc=%d", rc);
  const bool replace = flags & 1, relax = flags & 2;
  for (int64_t b = 0; b < B; ++b) {
    const int64_t* o = out.data() + b * (K + 1);
    if (relax) CHECK(label[o[0]] == tgt[b], "relax positive has the wrong class");
    else CHECK(o[0] == idx[b], "exact positive != index");
    std::set<int64_t> seen;
    for (int64_t k = 1; k <= K; ++k) {
      CHECK(o[k] >= 0 && o[k] < N, "negative out of range: %lld", (long long)o[k]);
      if (o[k] < 0 || o[k] >= N) continue;
      CHECK(label[o[k]] != tgt[b], "negative from the positive class");
      seen.insert(o[k]);
    }
    if (!replace && K <= N - count[tgt[b]])
      CHECK((int64_t)seen.size() == K, "duplicate negatives without replacement");
  }
}

static void alias_case(int64_t K) {
  std::vector<double> p(K);
  double tot = 0;
  for (int64_t i = 0; i < K; ++i) { p[i] = 1.0 + (i % 5); tot += p[i]; }
  std::vector<float> prob(K);
  std::vector<int64_t> alias(K);
  CHECK(mdah_alias_build(p.data(), prob.data(), alias.data(), K) == 0, "alias rc");
  // reconstructed probability of each outcome == p / tot
  std::vector<double> q(K, 0.0);
  for (int64_t i = 0; i < K; ++i) {
    CHECK(alias[i] >= 0 && alias[i] < K, "alias out of range");
    q[i] += prob[i] / K;
    q[alias[i]] += (1.0 - prob[i]) / K;
  }
  for (int64_t i = 0; i < K; ++i)
    CHECK(std::abs(q[i] - p[i] / tot) < 1e-5, "alias prob %lld: %g vs %g", (long long)i, q[i], p[i] / tot);
}

int main() {
  for (int64_t flags = 0; flags < 4; ++flags) {
    crd_case(1000, 10, 64, 200, flags);
    crd_case(50, 5, 16, 60, flags);   // K > #negatives: falls back to replacement
    crd_case(5000, 100, 128, 1024, flags);
  }
  alias_case(1);
  alias_case(17);
  alias_case(1000);
  if (g_fail) {
    fprintf(stderr, "%d check(s) failed\n", g_fail);
    return 1;
  }
  printf("host selftest ok\n");
  return 0;
}
