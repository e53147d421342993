// fastx_dump.cpp — host-only harness around nk::FastxReader (the CLI's and
// nk_process_file_streaming's parser) so its record semantics are testable
// without a GPU.  Prints JSON: {"rc":..,"err":..,"truncated":..,"records":[hex..]}.
// batch (argv[2], bases) exercises record batching across buffer refills.
// --mapped <window> <threads>: the host FASTQ extraction of the file ingest
// (nk_fqhost.h), window by window as nk_ingest_host.cpp runs it; prints
// "fallback" (a blank line where a header is due) instead of records then.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#include "neurokmer.h"
#include "nk_fastx.h"
#include "nk_fqhost.h"

static void print_records(const std::vector<uint8_t> &bases, const std::vector<uint64_t> &offs) {
  static const char *hx = "0123456789abcdef";
  for (size_t i = 0; i + 1 < offs.size(); ++i) {
    printf(i ? ",\"" : "\"");
    for (uint64_t p = offs[i]; p < offs[i + 1]; ++p) {
      putchar(hx[bases[p] >> 4]);
      putchar(hx[bases[p] & 15]);
    }
    putchar('"');
  }
}

static int mapped(const char *path, size_t win, int threads) {
  nk::MappedFile mf;
  std::string err;
  int rc = mf.open(path, err);
  std::vector<uint8_t> bases;
  std::vector<uint64_t> offs{0};
  bool stop = false, blank = false;
  if (!rc && !mf.size()) {
    rc = NK_E_PARSE;
    err = "empty file";
  }
  if (!rc && mf.data()[0] != '@') {
    rc = NK_E_PARSE;
    err = "not FASTQ";
  }
  if (!rc) {
    nk::HostPool pool(threads);
    std::vector<uint8_t> hb;
    std::vector<uint64_t> he;
    uint64_t pos = 0;
    for (;;) {
      const size_t len = (size_t)std::min<uint64_t>(win, mf.size() - pos);
      const bool eof = pos + len >= mf.size();
      hb.resize(len + 1);
      he.resize(nk::fq_max_records(len));
      nk::FqResult r = nk::fq_extract(mf.data() + pos, len, eof, hb.data(), he.data(), bases.size(), pool);
      if (!r.n_rec && !r.stop && !r.blank && !eof) {  // a record longer than the window
        win *= 2;
        continue;
      }
      bases.insert(bases.end(), hb.begin(), hb.begin() + r.n_bases);
      offs.insert(offs.end(), he.begin(), he.begin() + r.n_rec);
      pos += r.consumed;
      if (r.blank) { blank = true; break; }
      if (r.stop) { stop = true; break; }
      if (eof) break;
    }
  }
  printf("{\"rc\":%d,\"err\":\"%s\",\"truncated\":%s,\"fallback\":%s,\"records\":[", rc, err.c_str(),
         stop ? "true" : "false", blank ? "true" : "false");
  if (!blank) print_records(bases, offs);
  printf("]}\n");
  return 0;
}

int main(int argc, char **argv) {
  if (argc < 2) {
    fprintf(stderr, "usage: fastx_dump <file> [batch_bases | --mapped <window> <threads>]\n");
    return 2;
  }
  if (argc > 4 && !strcmp(argv[2], "--mapped"))
    return mapped(argv[1], strtoull(argv[3], nullptr, 10), atoi(argv[4]));
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
  print_records(bases, offs);
  printf("]}\n");
  return 0;
}
