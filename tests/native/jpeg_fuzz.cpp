// Mutation fuzz of the front end's baseline-JPEG -> coefficient-container decoder
// (frontend/csrc/jpeg_coefs.h) under AddressSanitizer + UndefinedBehaviorSanitizer: random byte
// flips and truncations of valid JPEGs must either decode or be refused, never read/write out of
// bounds.  Inputs: JPEG files on the command line (tests/test_native_sanitizers.py writes them).
#include <cstdio>
#include <fstream>
#include <iterator>
#include <random>
#include <vector>

#include "jpeg_coefs.h"

int main(int argc, char** argv) {
  std::vector<uint8_t> out(mlsjpeg::CONTAINER_BYTES);
  std::mt19937 rng(1);
  int ok = 0, refused = 0;
  for (int a = 1; a < argc; ++a) {
    std::ifstream f(argv[a], std::ios::binary);
    std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), {});
    if (d.size() < 4) return 2;
    std::string why;
    if (!mlsjpeg::jpeg_to_container(d.data(), d.size(), out.data(), &why)) return 3;  // the clean file decodes
    for (int it = 0; it < 2000; ++it) {
      std::vector<uint8_t> x = d;
      const int nm = 1 + (int)(rng() % 8);
      for (int k = 0; k < nm; ++k) x[2 + rng() % (x.size() - 2)] = (uint8_t)rng();
      if (it % 5 == 0) x.resize(2 + rng() % (x.size() - 2));
      (mlsjpeg::jpeg_to_container(x.data(), x.size(), out.data(), &why) ? ok : refused)++;
    }
  }
  std::printf("jpeg fuzz: ok (%d decoded, %d refused)\n", ok, refused);
  return 0;
}
