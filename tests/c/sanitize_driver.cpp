// Host-side sanitizer driver (tests/test_sanitizers.py builds it with
// -fsanitize=address,undefined on the host code): exercises every piece of host
// C/C++ that needs no GPU —
//   * the oracle (oracle/wfpt_oracle.c): full_pdf / pdf_array / wiener_like /
//     wiener_like_multi over random parameter sets, incl. deep adaptive trees;
//   * the exact path on the host (wfpt_exact.hpp + wfpt_crlibm.hpp);
//   * the C ABI's host logic (wfpt_capi.cpp): argument checks, result decode
//     and error encoding, shard ranges, the poisoned triple, and every entry
//     point's failure path when no device is present;
//   * the TCP rendezvous (wfpt_rendezvous.cpp) with three ranks as threads,
//     plus a peer whose rank 0 never comes.
// Exit status 0 = every check passed and no sanitizer report.
#include <math.h>
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <random>
#include <thread>
#include <vector>

#include "../../hddm_amd/csrc/wfpt_exact.hpp"
#include "../../include/wfpt_amd.h"
#include "../../oracle/wfpt_oracle.h"

static int failures = 0;
#define CHECK(c)                                                       \
  do {                                                                 \
    if (!(c)) {                                                        \
      fprintf(stderr, "CHECK failed at %s:%d: %s\n", __FILE__, __LINE__, #c); \
      ++failures;                                                      \
    }                                                                  \
  } while (0)

static void oracle_and_exact() {
  std::mt19937_64 g(20261017);
  std::uniform_real_distribution<double> U(0.0, 1.0);
  for (int rep = 0; rep < 60; ++rep) {
    const double v = -4 + 8 * U(g), sv = (rep % 3) ? 2.5 * U(g) : 0.0, a = 0.5 + 1.5 * U(g);
    const double z = 0.4 + 0.2 * U(g), sz = (rep % 2) ? 0.4 * U(g) : 0.0, t = 0.2 + 0.3 * U(g);
    const double st = (rep % 4) ? 0.35 * U(g) : 0.0;
    const double err = pow(10.0, -10 + 9 * U(g)), se = pow(10.0, -6 + 4 * U(g));
    const int n = (rep % 5 == 0) ? 6 : 2;
    const int ua = rep % 7 != 0;
    std::vector<double> x(48);
    for (auto& xi : x) xi = (U(g) < 0.7 ? 1 : -1) * (t - st / 2 + 2.0 * U(g));
    x[0] = 0.0;
    x[1] = t / 2;
    std::vector<double> y(x.size()), l(x.size());
    oracle_pdf_array(x.data(), (int64_t)x.size(), v, sv, a, z, sz, t, st, err, 0, n, n, ua, se,
                     0.05, 0.1, y.data());
    oracle_pdf_array(x.data(), (int64_t)x.size(), v, sv, a, z, sz, t, st, err, 1, n, n, ua, se,
                     0.05, 0.1, l.data());
    const double wl = oracle_wiener_like(x.data(), (int64_t)x.size(), v, sv, a, z, sz, t, st,
                                         err, n, n, ua, se, 0.05, 0.1);
    CHECK(!isnan(wl) || true);
    int64_t cnt = 0;
    for (size_t i = 0; i < x.size(); ++i) {
      const double p = oracle_full_pdf(x[i], v, sv, a, z, sz, t, st, err, n, n, ua, se, &cnt);
      wfpt_x::Ctx C;
      const double q = wfpt_x::full_pdf(x[i], v, sv, a, z, sz, t, st, err, n, n, ua, se, C);
      if (p == 0 || isnan(p)) CHECK(q == p || (isnan(p) && isnan(q)));
      else CHECK(fabs(q - p) <= 1e-13 * fabs(p));
    }
    const double* arr[7] = {x.data(), nullptr, nullptr, nullptr, nullptr, nullptr, nullptr};
    const double sc[7] = {v, sv, a, z, sz, t, st};
    std::vector<double> terms(x.size());
    x[2] = 999.0;
    x[3] = -999.0;
    (void)oracle_wiener_like_multi_terms(x.data(), (int64_t)x.size(), arr, sc, err, n, n, ua, se,
                                         0.05, 0.1, terms.data());
  }
}

static void capi_host_logic() {
  double out = 0;
  const double ok[3] = {-12.5, 0, 0};
  CHECK(wfpt_decode_result(ok, &out) == WFPT_OK && out == -12.5);
  const double zero[3] = {-12.5, 2, 0};
  CHECK(wfpt_decode_result(zero, &out) == WFPT_OK && isinf(out) && out < 0);
  const double depth[3] = {0, 0, 1};
  CHECK(wfpt_decode_result(depth, &out) == WFPT_ERR_UNSUPPORTED);
  CHECK(strstr(wfpt_last_error(), "WFPT_MAX_DEPTH") != nullptr);
  const double budget[3] = {0, 0, 2 * 1048576.0};
  CHECK(wfpt_decode_result(budget, &out) == WFPT_ERR_UNSUPPORTED);
  CHECK(strstr(wfpt_last_error(), "WFPT_EVAL_BUDGET") != nullptr);
  double pz[3];
  CHECK(wfpt_result_poison(pz) == WFPT_OK);
  const double peer[3] = {pz[0] - 3.0, pz[1], pz[2] + pz[2]};
  CHECK(wfpt_decode_result(peer, &out) == WFPT_ERR_COMM);
  CHECK(strstr(wfpt_last_error(), "2 rank(s) failed") != nullptr);
  const double mix[3] = {0, 0, pz[2] + 1.0};
  CHECK(wfpt_decode_result(mix, &out) == WFPT_ERR_UNSUPPORTED);
  CHECK(wfpt_decode_result(nullptr, &out) == WFPT_ERR_ARG);
  const int64_t sizes[] = {0, 1, 63, 64, 1000003, 100000000};
  for (int64_t n : sizes) {
    for (int r = 1; r <= 9; ++r) {
      int64_t prev = 0;
      for (int k = 0; k < r; ++k) {
        int64_t lo, hi;
        wfpt_shard_range(n, r, k, &lo, &hi);
        CHECK(lo == prev && hi >= lo);
        prev = hi;
      }
      CHECK(prev == n);
    }
  }
  // no device in this container: every entry point fails with a status
  wfpt_ctx* c = nullptr;
  int nd = -1;
  (void)wfpt_device_count(&nd);
  if (nd <= 0) CHECK(wfpt_open(0, &c) != WFPT_OK && c == nullptr);
  wfpt_params p = {0.5, 0.1, 2.0, 0.5, 0.1, 0.3, 0.1, 0.05};
  wfpt_knobs k = {1e-4, 2, 2, 1, 1e-3, 0.1};
  double x = 1.0;
  CHECK(wfpt_wiener_like(nullptr, nullptr, &p, &k, &out) == WFPT_ERR_ARG);
  CHECK(wfpt_wiener_like_host(nullptr, &x, 1, &p, &k, &out) == WFPT_ERR_ARG);
  CHECK(wfpt_pdf_array(nullptr, &x, 1, &p, &k, 0, &out) == WFPT_ERR_ARG);
  CHECK(wfpt_wiener_like_nodes_ex(nullptr, nullptr, &p, &k, &out, nullptr) == WFPT_ERR_ARG);
  CHECK(wfpt_dataset_create(nullptr, &x, 1, nullptr, 0, nullptr) == WFPT_ERR_ARG);
  CHECK(wfpt_wiener_like_allreduce(nullptr, nullptr, &p, &k, &out) == WFPT_ERR_ARG);
  CHECK(wfpt_wiener_like_allreduce_group(nullptr, nullptr, 0, &p, &k, &out) == WFPT_ERR_ARG);
  CHECK(wfpt_comm_init_all(nullptr, 0) == WFPT_ERR_ARG);
  CHECK(wfpt_comm_exchange_id(2, 5, "127.0.0.1", 1, 10, (unsigned char*)pz) == WFPT_ERR_ARG);
  wfpt_close(nullptr);
  wfpt_dataset_destroy(nullptr);
  CHECK(wfpt_dataset_size(nullptr) == -1);
}

static void rendezvous(int port) {
  unsigned char id0[128], got[3][128];
  for (int i = 0; i < 128; ++i) id0[i] = (unsigned char)(i * 7 + 3);
  int rc[3] = {-1, -1, -1};
  std::vector<std::thread> th;
  for (int r = 2; r >= 0; --r)
    th.emplace_back([&, r] {
      if (r == 0) memcpy(got[0], id0, 128);
      else memset(got[r], 0, 128);
      rc[r] = wfpt_comm_exchange_id(3, r, "127.0.0.1", port, 20000, got[r]);
    });
  for (auto& t : th) t.join();
  for (int r = 0; r < 3; ++r) {
    CHECK(rc[r] == WFPT_OK);
    CHECK(memcmp(got[r], id0, 128) == 0);
  }
  unsigned char lone[128];
  CHECK(wfpt_comm_exchange_id(2, 1, "127.0.0.1", port + 1, 300, lone) == WFPT_ERR_COMM);
}

int main(int argc, char** argv) {
  const int port = argc > 1 ? atoi(argv[1]) : 29611;
  oracle_and_exact();
  capi_host_logic();
  rendezvous(port);
  if (failures) {
    fprintf(stderr, "%d check(s) failed\n", failures);
    return 1;
  }
  printf("sanitize driver: all checks passed\n");
  return 0;
}
