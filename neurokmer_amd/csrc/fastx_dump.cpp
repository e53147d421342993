// fastx_dump.cpp — host-only harness around nk::FastxReader (the CLI's and
// nk_process_file_streaming's parser) so its record semantics are testable
// without a GPU.  Prints JSON: {"rc":..,"err":..,"truncated":..,"records":[hex..]}.
// batch (argv[2], bases) exercises record batching across buffer refills.
#include <stdio.h>
#include <stdlib.h>

#include <string>
#include <vector>

#include "nk_fastx.h"

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: fastx_dump <file> [batch_bases]\n");
    return 2;
  }
  size_t batch = argc > 2 ? strtoull(argv[2], nullptr, 10) : (1u << 20);
  nk::FastxReader r;
  std::string err;
  int rc = r.open(argv[1], err);
  std::vector<uint8_t> bases;
  std::vector<uint64_t> offs{0};
  if (!rc)
    while (r.next_batch(batch, bases, offs)) {
    }
  printf("{\"rc\":%d,\"err\":\"%s\",\"truncated\":%s,\"records\":[", rc, err.c_str(),
         r.truncated() ? "true" : "false");
  static const char *hx = "0123456789abcdef";
  for (size_t i = 0; i + 1 < offs.size(); ++i) {
    printf(i ? ",\"" : "\"");
    for (uint64_t p = offs[i]; p < offs[i + 1]; ++p) {
      putchar(hx[bases[p] >> 4]);
      putchar(hx[bases[p] & 15]);
    }
    putchar('"');
  }
  printf("]}\n");
  return 0;
}
