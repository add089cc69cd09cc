// Host build of ragen_amd/csrc/pyrepr.hpp (TEST INFRASTRUCTURE): reads doubles (f64 LE) from
// argv[1], writes one line per value — py_float_repr's text, or "?" where it returns -1.
#include <cstdio>
#include <vector>

#include "../../ragen_amd/csrc/pyrepr.hpp"

int main(int argc, char** argv) {
  if (argc != 3) return 2;
  std::FILE* f = std::fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<double> xs;
  double x;
  while (std::fread(&x, sizeof x, 1, f) == 1) xs.push_back(x);
  std::fclose(f);
  std::FILE* o = std::fopen(argv[2], "w");
  if (!o) return 2;
  char buf[64], scratch[64];
  for (double v : xs) {
    const int n = rmi::py_float_repr(v, buf, scratch);
    if (n < 0) {
      std::fputs("?\n", o);
    } else {
      std::fwrite(buf, 1, n, o);
      std::fputc('\n', o);
    }
  }
  std::fclose(o);
  return 0;
}
