// Host build of the exact path (hddm_amd/csrc/wfpt_exact.hpp) for
// tests/test_exact_path.py: per-trial full_pdf, compared with the oracle.
#include <stdint.h>
#include "../../hddm_amd/csrc/wfpt_exact.hpp"
extern "C" void exact_pdf_array(const double* x, int64_t n, double v, double sv, double a,
                                double z, double sz, double t, double st, double err, int n_st,
                                int n_sz, int use_adaptive, double simps_err, double* out) {
  for (int64_t i = 0; i < n; ++i) {
    wfpt_x::Ctx C;
    out[i] = wfpt_x::full_pdf(x[i], v, sv, a, z, sz, t, st, err, n_st, n_sz, use_adaptive,
                              simps_err, C);
  }
}
