// Host check of hddm_amd/csrc/wfpt_crlibm.hpp (tests/test_crlibm.py):
// reads doubles (function id, x) from stdin-less generated streams and prints
// the cr_* result and glibc's result as hex bit patterns.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include "../../hddm_amd/csrc/wfpt_crlibm.hpp"
using namespace wfpt_cr;
int main(int argc, char** argv) {
  // argv[1]: input file of doubles (x), argv[2]: fn id, argv[3]: output file
  FILE* f = fopen(argv[1], "rb");
  int fn = atoi(argv[2]);
  FILE* o = fopen(argv[3], "wb");
  double x;
  while (fread(&x, 8, 1, f) == 1) {
    double c, g;
    switch (fn) {
      case 0: c = cr_exp(x); g = exp(x); break;
      case 1: c = cr_log(x); g = log(x); break;
      case 2: c = cr_sin(x); g = sin(x); break;
      default: c = cr_cube(x); g = pow(x, 3.0); break;
    }
    fwrite(&c, 8, 1, o);
    fwrite(&g, 8, 1, o);
  }
  fclose(o);
  fclose(f);
  return 0;
}
