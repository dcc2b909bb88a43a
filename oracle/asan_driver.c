/*
 * asan_driver.c — the oracle's C restatement under AddressSanitizer + UBSan (TEST
 * INFRASTRUCTURE, SURVEY.md §5 "ASan/UBSan on the CPU build").  `make -C oracle asan`
 * builds oracle.c and this driver with -fsanitize=address,undefined and runs it: every
 * exported function on edge-case and random inputs (empty graphs, rows of degree 0, one
 * row holding every edge, a row above the heavy-row split, fanouts 0 / 1 / 64 / above the
 * degree, exclusions, Zipf), each result checked against a naive restatement here.  Any
 * sanitizer report aborts with a non-zero status.
 */
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

uint64_t oracle_hash3(uint64_t seed, uint64_t a, uint64_t b);
int oracle_num_threads(void);
void oracle_spmm_csr_f32(const int64_t* indptr, const int32_t* indices, const float* ew,
                         const float* X, int64_t ldx, int64_t n_dst, int64_t d, int reduce,
                         float* out, int64_t ldo);
void oracle_spmm_csr_f64acc(const int64_t* indptr, const int32_t* indices, const float* ew,
                            const float* X, int64_t ldx, int64_t n_dst, int64_t d, int mean,
                            float* out, int64_t ldo);
void oracle_synth_edges(uint64_t seed, int64_t e0, int64_t n, int64_t n_u, int64_t n_i,
                        const double* cdf, int32_t* u, int32_t* it);
void oracle_fill_f32(uint64_t seed, int64_t n, float* out);
void oracle_sample_count(const int64_t* indptr, const int64_t* eids, const uint8_t* excluded,
                         const int64_t* seeds, int64_t n_seeds, int64_t fanout, uint64_t key,
                         int64_t* counts);
void oracle_sample_fill(const int64_t* indptr, const int64_t* indices, const int64_t* eids,
                        const uint8_t* excluded, const int64_t* seeds, int64_t n_seeds,
                        int64_t fanout, uint64_t key, const int64_t* out_indptr, int64_t* out_src,
                        int64_t* out_eid);
void oracle_csr_from_coo(const int64_t* src, const int64_t* dst, int64_t E, int64_t n_dst,
                         int64_t* indptr, int32_t* indices, int64_t* eids);

static int g_fail = 0;
#define CHECK(c, ...)                                  \
  do {                                                 \
    if (!(c)) {                                        \
      fprintf(stderr, "FAIL %s:%d: ", __FILE__, __LINE__); \
      fprintf(stderr, __VA_ARGS__);                    \
      fprintf(stderr, "\n");                           \
      g_fail = 1;                                      \
    }                                                  \
  } while (0)

static uint64_t rng_state = 0x1234567ull;
static uint64_t rnd(void) {
  rng_state ^= rng_state << 13;
  rng_state ^= rng_state >> 7;
  rng_state ^= rng_state << 17;
  return rng_state;
}

static void* xmalloc(size_t n) {
  void* p = malloc(n ? n : 1);
  if (!p) abort();
  return p;
}

/* a COO graph -> CSR by the oracle, checked against a naive counting pass */
static void build(int64_t E, int64_t n_src, int64_t n_dst, int64_t* src, int64_t* dst,
                  int64_t* indptr, int32_t* indices, int64_t* eids) {
  oracle_csr_from_coo(src, dst, E, n_dst, indptr, indices, eids);
  CHECK(indptr[0] == 0 && indptr[n_dst] == E, "csr: indptr ends %lld", (long long)indptr[n_dst]);
  int64_t* cnt = xmalloc(sizeof(int64_t) * (size_t)(n_dst + 1));
  memset(cnt, 0, sizeof(int64_t) * (size_t)(n_dst + 1));
  for (int64_t e = 0; e < E; ++e) cnt[dst[e]]++;
  for (int64_t r = 0; r < n_dst; ++r) {
    CHECK(indptr[r + 1] - indptr[r] == cnt[r], "csr: row %lld degree", (long long)r);
    for (int64_t k = indptr[r]; k < indptr[r + 1]; ++k) {
      const int64_t e = eids[k];
      CHECK(dst[e] == r && src[e] == indices[k], "csr: edge %lld misplaced", (long long)e);
      if (k > indptr[r]) CHECK(eids[k - 1] < e, "csr: row %lld not in eid order", (long long)r);
    }
  }
  (void)n_src;
  free(cnt);
}

static void check_spmm(const int64_t* indptr, const int32_t* indices, int64_t n_dst, int64_t n_src,
                       int64_t d) {
  float* X = xmalloc(sizeof(float) * (size_t)(n_src * d));
  oracle_fill_f32(7, n_src * d, X);
  for (int64_t i = 0; i < n_src * d; ++i) CHECK(X[i] >= -1.f && X[i] < 1.f, "fill range");
  const int64_t E = indptr[n_dst];
  float* ew = xmalloc(sizeof(float) * (size_t)E);
  for (int64_t e = 0; e < E; ++e) ew[e] = (float)(1 + rnd() % 8);
  float* out = xmalloc(sizeof(float) * (size_t)(n_dst * d));
  float* ref = xmalloc(sizeof(float) * (size_t)d);
  for (int reduce = 0; reduce < 3; ++reduce) {
    for (int w = 0; w < 2; ++w) {
      oracle_spmm_csr_f32(indptr, indices, w ? ew : NULL, X, d, n_dst, d, reduce, out, d);
      for (int64_t v = 0; v < n_dst; v += 1 + (int64_t)(rnd() % 7)) {
        const int64_t deg = indptr[v + 1] - indptr[v];
        for (int64_t c = 0; c < d; ++c) ref[c] = reduce == 2 ? -INFINITY : 0.f;
        for (int64_t k = indptr[v]; k < indptr[v + 1]; ++k)
          for (int64_t c = 0; c < d; ++c) {
            const float m = X[(int64_t)indices[k] * d + c] * (w ? ew[k] : 1.f);
            if (reduce == 2) ref[c] = m > ref[c] ? m : ref[c];
            else ref[c] += m;
          }
        for (int64_t c = 0; c < d; ++c) {
          float r = ref[c];
          if (reduce == 1) r = r / (float)(deg > 0 ? deg : 1);
          if (reduce == 2 && deg == 0) r = 0.f;
          CHECK(out[v * d + c] == r, "spmm reduce %d w %d row %lld col %lld: %g vs %g", reduce, w,
                (long long)v, (long long)c, out[v * d + c], r);
        }
      }
    }
    if (reduce < 2) {  /* the double accumulator: close to the fp32 sum on small rows */
      oracle_spmm_csr_f64acc(indptr, indices, NULL, X, d, n_dst, d, reduce, out, d);
      float* o32 = xmalloc(sizeof(float) * (size_t)(n_dst * d));
      oracle_spmm_csr_f32(indptr, indices, NULL, X, d, n_dst, d, reduce, o32, d);
      for (int64_t i = 0; i < n_dst * d; ++i)
        CHECK(fabsf(out[i] - o32[i]) <= 1e-3f * (1.f + fabsf(o32[i])) + 1e-2f, "f64acc %lld",
              (long long)i);
      free(o32);
    }
  }
  free(X);
  free(ew);
  free(out);
  free(ref);
}

static void check_sampler(const int64_t* indptr, const int32_t* indices32, const int64_t* eids,
                          int64_t n_dst, int64_t E) {
  int64_t* indices = xmalloc(sizeof(int64_t) * (size_t)E);
  for (int64_t e = 0; e < E; ++e) indices[e] = indices32[e];
  uint8_t* excl = xmalloc((size_t)E);
  for (int64_t e = 0; e < E; ++e) excl[e] = (uint8_t)(rnd() % 5 == 0);
  const int64_t n_seeds = n_dst < 300 ? n_dst : 300;
  int64_t* seeds = xmalloc(sizeof(int64_t) * (size_t)n_seeds);
  for (int64_t i = 0; i < n_seeds; ++i) seeds[i] = (int64_t)(rnd() % (uint64_t)n_dst);
  const int64_t fans[] = {-1, 0, 1, 3, 10, 64};
  int64_t* counts = xmalloc(sizeof(int64_t) * (size_t)n_seeds);
  int64_t* ip = xmalloc(sizeof(int64_t) * (size_t)(n_seeds + 1));
  for (size_t f = 0; f < sizeof(fans) / sizeof(fans[0]); ++f) {
    for (int x = 0; x < 2; ++x) {
      const uint8_t* ex = x ? excl : NULL;
      oracle_sample_count(indptr, eids, ex, seeds, n_seeds, fans[f], 99 + f, counts);
      ip[0] = 0;
      for (int64_t i = 0; i < n_seeds; ++i) ip[i + 1] = ip[i] + counts[i];
      int64_t* os = xmalloc(sizeof(int64_t) * (size_t)ip[n_seeds]);
      int64_t* oe = xmalloc(sizeof(int64_t) * (size_t)ip[n_seeds]);
      oracle_sample_fill(indptr, indices, eids, ex, seeds, n_seeds, fans[f], 99 + f, ip, os, oe);
      for (int64_t i = 0; i < n_seeds; ++i) {
        const int64_t v = seeds[i], deg = indptr[v + 1] - indptr[v];
        const int64_t want = fans[f] < 0 || deg <= fans[f] ? deg : fans[f];
        CHECK(counts[i] <= want, "sampler: too many picks");
        if (!ex) CHECK(counts[i] == want, "sampler: count %lld vs %lld", (long long)counts[i],
                       (long long)want);
        for (int64_t k = ip[i]; k < ip[i + 1]; ++k) {
          int found = 0;
          for (int64_t q = indptr[v]; q < indptr[v + 1]; ++q)
            found |= eids[q] == oe[k] && indices[q] == os[k];
          CHECK(found, "sampler: pick is not an in-edge of its seed");
          CHECK(!ex || !ex[oe[k]], "sampler: excluded edge kept");
          if (k > ip[i]) CHECK(oe[k - 1] < oe[k], "sampler: picks not distinct / ordered");
        }
      }
      free(os);
      free(oe);
    }
  }
  free(indices);
  free(excl);
  free(seeds);
  free(counts);
  free(ip);
}

static void graph_case(const char* name, int64_t n_src, int64_t n_dst, int64_t E, int mode,
                       int64_t d) {
  int64_t* src = xmalloc(sizeof(int64_t) * (size_t)E);
  int64_t* dst = xmalloc(sizeof(int64_t) * (size_t)E);
  for (int64_t e = 0; e < E; ++e) {
    src[e] = (int64_t)(rnd() % (uint64_t)n_src);
    dst[e] = mode == 1 ? n_dst - 1 : (int64_t)(rnd() % (uint64_t)n_dst);  /* 1: one row */
  }
  int64_t* indptr = xmalloc(sizeof(int64_t) * (size_t)(n_dst + 1));
  int32_t* indices = xmalloc(sizeof(int32_t) * (size_t)E);
  int64_t* eids = xmalloc(sizeof(int64_t) * (size_t)E);
  build(E, n_src, n_dst, src, dst, indptr, indices, eids);
  check_spmm(indptr, indices, n_dst, n_src, d);
  if (E < 200000) check_sampler(indptr, indices, eids, n_dst, E);
  fprintf(stderr, "ok %s\n", name);
  free(src);
  free(dst);
  free(indptr);
  free(indices);
  free(eids);
}

int main(void) {
  /* the generator: uniform and Zipf, chunks regenerate the same stream */
  {
    const int64_t n = 100000, nu = 1000, ni = 300;
    int32_t *u = xmalloc(4 * n), *it = xmalloc(4 * n), *u2 = xmalloc(4 * n), *i2 = xmalloc(4 * n);
    double* cdf = xmalloc(sizeof(double) * ni);
    double s = 0;
    for (int64_t j = 0; j < ni; ++j) s += 1.0 / (double)(j + 1);
    double acc = 0;
    for (int64_t j = 0; j < ni; ++j) cdf[j] = (acc += 1.0 / (double)(j + 1) / s);
    cdf[ni - 1] = 1.0;
    for (int z = 0; z < 2; ++z) {
      oracle_synth_edges(11, 0, n, nu, ni, z ? cdf : NULL, u, it);
      oracle_synth_edges(11, 40000, n - 40000, nu, ni, z ? cdf : NULL, u2, i2);
      for (int64_t k = 0; k < n; ++k) {
        CHECK(u[k] >= 0 && u[k] < nu && it[k] >= 0 && it[k] < ni, "synth range");
        if (k >= 40000) CHECK(u[k] == u2[k - 40000] && it[k] == i2[k - 40000], "synth chunks");
      }
    }
    free(u);
    free(it);
    free(u2);
    free(i2);
    free(cdf);
    fprintf(stderr, "ok synth (%d threads)\n", oracle_num_threads());
  }
  graph_case("empty graph", 5, 7, 0, 0, 4);
  graph_case("single dst row", 50, 1, 2000, 0, 3);
  graph_case("ragged random", 400, 300, 6000, 0, 16);
  graph_case("every edge into one row", 200, 90, 5000, 1, 8);
  graph_case("heavy row above the column split", 64, 2, (1 << 20) + 777, 1, 8);
  return g_fail;
}
