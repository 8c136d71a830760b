// Host-only driver of the product's ONNX loader (onnx_model.cpp: parse_onnx and the
// inspect_json view behind go2pi_inspect_model) for the sanitizer fuzz test
// (tests/test_cpu_fuzz.py, built with -fsanitize=address,undefined). Every file
// named on the command line is parsed; a malformed one must end in a clean
// std::exception (the C ABI maps it to GO2PI_E_MODEL), never in a crash or a
// sanitizer report. Prints one line per file: "ok <json bytes>" or "error <what>".
#include <cstdio>
#include <exception>
#include <fstream>
#include <iterator>
#include <string>
#include <vector>

#include "onnx_model.hpp"

int main(int argc, char **argv) {
  for (int i = 1; i < argc; ++i) {
    std::ifstream f(argv[i], std::ios::binary);
    std::vector<uint8_t> bytes((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    try {
      const go2pi::Model m = go2pi::parse_onnx(bytes.data(), bytes.size());
      std::printf("ok %zu\n", go2pi::inspect_json(m).size());
    } catch (const std::exception &ex) {
      std::string w = ex.what();  // (names from the file: one line, printable)
      for (char &c : w)
        if ((unsigned char)c < 0x20 || (unsigned char)c >= 0x7F) c = '?';
      std::printf("error %s\n", w.c_str());
    }
  }
  return 0;
}
