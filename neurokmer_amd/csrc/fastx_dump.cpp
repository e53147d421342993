// fastx_dump.cpp — host-only harness around nk::FastxReader (the CLI's and
// nk_process_file_streaming's parser) so its record semantics are testable
// without a GPU.  Prints JSON: {"rc":..,"err":..,"truncated":..,"records":[hex..]}.
// batch (argv[2], bases) exercises record batching across buffer refills.
// --mapped <window> <threads> [max_rec]: the host FASTQ extraction of the file ingest
// (nk_fqhost.h: threads pread and parse), window by window as
// nk_ingest_host.cpp runs it; prints
// "fallback" (a blank line where a header is due) instead of records then.
// --shrink <bytes> after --mapped's arguments: the file is cut to that size
// after it was opened and sized (a read that ends early: NK_E_IO, not a stop).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

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

static int mapped(const char *path, size_t win, int threads, uint64_t max_rec, long long shrink) {
  nk::HostFile hf;
  std::string err;
  int rc = hf.open(path, err);
  if (!rc && shrink >= 0 && truncate(path, (off_t)shrink) != 0) {
    rc = NK_E_IO;
    err = "truncate failed";
  }
  std::vector<uint8_t> bases;
  std::vector<uint64_t> offs{0};
  bool stop = false, blank = false;
  uint8_t b0 = 0;
  if (!rc && !hf.size()) {
    rc = NK_E_PARSE;
    err = "empty file";
  }
  if (!rc && (pread(hf.fd(), &b0, 1, 0) != 1 || b0 != '@')) {
    rc = NK_E_PARSE;
    err = "not FASTQ";
  }
  if (!rc) {
    nk::HostPool pool(threads);
    std::vector<uint8_t> rb, hb;
    std::vector<uint64_t> he;
    uint64_t pos = 0;
    for (;;) {
      const size_t len = (size_t)std::min<uint64_t>(win, hf.size() - pos);
      const bool eof = pos + len >= hf.size();
      rb.resize(len + 64);
      hb.resize(len + 1);
      he.resize(nk::fq_max_records(len));
      nk::FqResult r = nk::fq_extract(rb.data(), len, eof, hb.data(), he.data(), bases.size(), pool,
                                      hf.fd(), pos, nullptr, max_rec);
      if (!r.io_error.empty()) {  // (nk_ingest_host.cpp: NK_E_IO)
        rc = NK_E_IO;
        err = r.io_error;
        break;
      }
      if (!r.n_rec && !r.stop && !r.blank && !eof) {  // a record longer than the window
        win *= 2;
        continue;
      }
      bases.insert(bases.end(), hb.begin(), hb.begin() + r.n_bases);
      offs.insert(offs.end(), he.begin(), he.begin() + r.n_rec);
      pos += r.consumed;
      if (r.blank) { blank = true; break; }
      if (r.stop) {
        nk::warn_malformed(path, offs.size() - 1, "a FASTQ record is malformed or cut off");
        stop = true;
        break;
      }
      if (eof && !r.more) break;
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
  if (argc > 4 && !strcmp(argv[2], "--mapped")) {
    long long shrink = -1;
    uint64_t max_rec = ~0ull;
    for (int i = 5; i < argc; ++i) {
      if (!strcmp(argv[i], "--shrink") && i + 1 < argc) shrink = atoll(argv[++i]);
      else max_rec = strtoull(argv[i], nullptr, 10);
    }
    return mapped(argv[1], strtoull(argv[3], nullptr, 10), atoi(argv[4]), max_rec, shrink);
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
  if (!rc && r.io_error()) {
    rc = NK_E_IO;
    err = r.io_why();
  }
  printf("{\"rc\":%d,\"err\":\"%s\",\"truncated\":%s,\"records\":[", rc, err.c_str(),
         r.truncated() ? "true" : "false");
  print_records(bases, offs);
  printf("]}\n");
  return 0;
}
