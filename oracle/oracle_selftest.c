/* TEST INFRASTRUCTURE ONLY: a standalone driver for the host
 * AddressSanitizer / UBSan build of the oracle (`make -C oracle asan`,
 * sanitizers on host code).  Runs every oracle entry point on
 * small random multigraphs (empty rows, isolated nodes, self-loops,
 * multi-edges, E = 0, N = 1) and checks known answers that hold for any
 * graph:
 *   - sum aggregation of all-ones features = in-degree, mean = 1 on non-empty rows;
 *   - max of all-ones = 1 on non-empty rows, 0 (fill fix-up) on empty ones;
 *   - the adjoint of the sum with dZ = 1 is the out-degree;
 *   - 'sm' weights of a symmetric graph are symmetric per edge pair.
 * Exit status 0 = all checks passed (the sanitizers abort on any error). */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>

void oracle_degnorm(int64_t, int64_t, const int64_t *, const int64_t *, const float *,
                    const float *, int, float *, float *, float *);
void oracle_aggr_fwd(int64_t, int64_t, int64_t, const int64_t *, const int64_t *, const float *,
                     const float *, int, const float *, int, float *, int64_t *);
void oracle_aggr_bwd(int64_t, int64_t, int64_t, int64_t, const int64_t *, const int64_t *,
                     const float *, const float *, int, const float *, const float *, int,
                     const int64_t *, float *, float *);
void oracle_segment_mean(int64_t, int64_t, const int64_t *, const float *, float *);

static uint64_t rng = 88172645463325252ull;
static int64_t rnd(int64_t n) {
  rng ^= rng << 13;
  rng ^= rng >> 7;
  rng ^= rng << 17;
  return (int64_t)(rng % (uint64_t)n);
}

static int fails = 0;
#define CHECK(c, ...)                     \
  do {                                    \
    if (!(c)) {                           \
      fprintf(stderr, __VA_ARGS__);       \
      fputc('\n', stderr);                \
      ++fails;                            \
    }                                     \
  } while (0)

static void one_graph(int64_t N, int64_t pairs, int64_t F, int isolated) {
  const int64_t active = N - isolated > 0 ? N - isolated : 1;
  const int64_t E = 2 * pairs + N;
  int64_t *src = malloc(sizeof(int64_t) * (size_t)(E + 1));
  int64_t *dst = malloc(sizeof(int64_t) * (size_t)(E + 1));
  for (int64_t k = 0; k < pairs; ++k) {
    const int64_t s = rnd(active), d = rnd(active);
    src[2 * k] = s, dst[2 * k] = d;
    src[2 * k + 1] = d, dst[2 * k + 1] = s;
  }
  for (int64_t i = 0; i < N; ++i) src[2 * pairs + i] = dst[2 * pairs + i] = i;
  const size_t nf = (size_t)(N * F > 0 ? N * F : 1);
  float *ones = malloc(sizeof(float) * nf), *Y = malloc(sizeof(float) * nf);
  float *dH = malloc(sizeof(float) * nf), *db = malloc(sizeof(float) * (size_t)F);
  int64_t *am = malloc(sizeof(int64_t) * nf);
  float *deg = malloc(sizeof(float) * (size_t)N), *dinv = malloc(sizeof(float) * (size_t)N);
  float *norm = malloc(sizeof(float) * (size_t)(E + 1));
  int64_t *indeg = calloc((size_t)N, sizeof(int64_t)), *outdeg = calloc((size_t)N, sizeof(int64_t));
  for (size_t i = 0; i < nf; ++i) ones[i] = 1.0f;
  for (int64_t e = 0; e < E; ++e) ++indeg[dst[e]], ++outdeg[src[e]];

  oracle_degnorm(N, E, src, dst, NULL, NULL, 1, deg, dinv, norm);
  for (int64_t k = 0; k < pairs; ++k)
    CHECK(norm[2 * k] == norm[2 * k + 1], "sm weights not symmetric at pair %lld", (long long)k);
  for (int red = 0; red < 3; ++red) {
    oracle_aggr_fwd(N, E, F, src, dst, ones, NULL, red, NULL, 0, Y, red == 2 ? am : NULL);
    for (int64_t i = 0; i < N; ++i) {
      const float want = red == 0 ? (float)indeg[i] : (indeg[i] ? 1.0f : 0.0f);
      CHECK(Y[i * F] == want, "reduce %d row %lld: %g != %g", red, (long long)i, Y[i * F], want);
    }
  }
  oracle_aggr_bwd(N, N, E, F, src, dst, NULL, NULL, 0, ones, NULL, 0, NULL, dH, db);
  for (int64_t i = 0; i < N; ++i)
    CHECK(dH[i * F] == (float)outdeg[i], "adjoint row %lld", (long long)i);
  oracle_aggr_fwd(N, E, F, src, dst, ones, norm, 2, ones, 1, Y, am);
  oracle_aggr_bwd(N, N, E, F, src, dst, norm, dinv, 2, ones, Y, 1, am, dH, db);
  oracle_aggr_bwd(N, N, E, F, src, dst, norm, NULL, 1, ones, Y, 1, NULL, dH, db);
  int64_t ptr[4] = {0, N / 3, N / 3, N};
  float seg[3 * 64];
  if (F <= 64) oracle_segment_mean(3, F, ptr, ones, seg);
  free(src), free(dst), free(ones), free(Y), free(dH), free(db), free(am), free(deg), free(dinv);
  free(norm), free(indeg), free(outdeg);
}

int main(void) {
  one_graph(1, 0, 3, 0);
  one_graph(17, 0, 5, 0);
  one_graph(500, 2000, 16, 40);
  one_graph(301, 900, 64, 0);
  one_graph(64, 5000, 7, 3);
  if (fails) {
    fprintf(stderr, "oracle self-test: %d failures\n", fails);
    return 1;
  }
  printf("oracle self-test: ok\n");
  return 0;
}
