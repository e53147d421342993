// nk_cli.cpp — `neurokmer` CLI, the MI355X drop-in for the reference binary
// (src/main.rs:9-77).  Same flags (-i/--input, -k/--k [31], --pool-size
// [1000000], --canonical, --streaming), same LIF constants (threshold 1.0,
// leak 0.95, refractory 2, spike_cost 1.0: src/main.rs:36-37) and the same
// result block on stdout (src/main.rs:49-74).  Uses only the C ABI.
#include <charconv>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <string>
#include <vector>

#include "neurokmer.h"
#include "nk_fastx.h"

// Rust `{}` for f64: shortest round-trip digits in positional notation.
static std::string rust_f64(double x) {
  if (x != x) return "NaN";
  if (x == 1.0 / 0.0) return "inf";
  if (x == -1.0 / 0.0) return "-inf";
  char buf[512];
  auto res = std::to_chars(buf, buf + sizeof buf, x, std::chars_format::fixed);
  std::string s(buf, res.ptr);
  return s;
}

static void usage() {
  fprintf(stderr,
          "Neuromorphic k-mer counting with fixed-size spiking neuron pool\n\n"
          "Usage: neurokmer [OPTIONS] --input <INPUT>\n\n"
          "Options:\n"
          "  -i, --input <INPUT>\n"
          "  -k, --k <K>                  [default: 31]\n"
          "      --pool-size <POOL_SIZE>  [default: 1000000]\n"
          "      --canonical\n"
          "      --streaming\n"
          "      --device <N>             HIP device ordinal [default: 0]\n"
          "  -h, --help                   Print help\n");
}

static bool parse_u64(const char *s, unsigned long long &out) {
  char *end = nullptr;
  if (!s || !*s || *s == '-') return false;
  out = strtoull(s, &end, 10);
  return end && *end == 0;
}

int main(int argc, char **argv) {
  std::string input;
  unsigned long long k = 31, pool = 1000000, device = 0;
  bool canonical = false, streaming = false, have_input = false;
  for (int i = 1; i < argc; ++i) {
    std::string a = argv[i];
    auto val = [&](const char *name) -> const char * {
      size_t eq = a.find('=');
      if (eq != std::string::npos) return argv[i] + eq + 1;
      if (i + 1 >= argc) {
        fprintf(stderr, "error: a value is required for '%s'\n", name);
        exit(2);
      }
      return argv[++i];
    };
    auto is = [&](const char *opt) {
      return a == opt || a.rfind(std::string(opt) + "=", 0) == 0;
    };
    if (a == "-h" || a == "--help") {
      usage();
      return 0;
    } else if (a == "-i" || is("--input")) {
      input = val("--input <INPUT>");
      have_input = true;
    } else if (a == "-k" || is("--k")) {
      if (!parse_u64(val("--k <K>"), k)) { fprintf(stderr, "error: invalid value for '--k <K>'\n"); return 2; }
    } else if (is("--pool-size")) {
      if (!parse_u64(val("--pool-size <POOL_SIZE>"), pool)) { fprintf(stderr, "error: invalid value for '--pool-size <POOL_SIZE>'\n"); return 2; }
    } else if (a == "--canonical") {
      canonical = true;
    } else if (a == "--streaming") {
      streaming = true;
    } else if (is("--device")) {
      if (!parse_u64(val("--device <N>"), device)) { fprintf(stderr, "error: invalid value for '--device <N>'\n"); return 2; }
    } else {
      fprintf(stderr, "error: unexpected argument '%s' found\n", a.c_str());
      usage();
      return 2;
    }
  }
  if (!have_input) {
    fprintf(stderr, "error: the following required arguments were not provided:\n  --input <INPUT>\n");
    usage();
    return 2;
  }
  fprintf(stderr, "[INFO neurokmer] Starting NeuroKmer on %s (k=%llu, pool_size=%llu, canonical=%s, streaming=%s)\n",
          input.c_str(), k, pool, canonical ? "true" : "false", streaming ? "true" : "false");

  nk_opts opts;
  nk_opts_default(&opts);
  opts.device = (int32_t)device;
  nk_counter *c = nk_new((size_t)k, 1.0f, 0.95f, 2, 1.0, (size_t)pool, canonical ? 1 : 0, &opts);
  if (!c) {
    fprintf(stderr, "Error: %s\n", nk_last_error());
    return 1;
  }
  int rc;
  if (streaming) {
    printf("Starting streaming for: %s\n", input.c_str());
    rc = nk_process_file_streaming(c, input.c_str());
  } else {
    // stream_sequences(input).collect() + process_parallel (src/main.rs:40-46),
    // parsed on the device (nk_process_file_parallel)
    rc = nk_process_file_parallel(c, input.c_str());
    if (!rc) {
      std::vector<uint64_t> cur(nk_pool_size(c));
      unsigned long long tot = 0;
      if (!cur.empty() && nk_copy_currents(c, cur.data(), cur.size()) == 0)
        for (uint64_t x : cur) tot += x;
      printf("  In-memory total current: %llu\n", tot);  // src/spiking_hash.rs:184
    }
  }
  if (rc) {
    fprintf(stderr, "Error: %s\n", nk_last_error());
    nk_free(c);
    return 1;
  }
  printf("\n=== Top 20 Abundant Neuron Groups (Highest Spike Rates) ===\n");
  std::vector<nk_top_row> top(20);
  long n = nk_top_abundant_neurons(c, 20, top.data());
  if (n < 0) {
    fprintf(stderr, "Error: %s\n", nk_last_error());
    nk_free(c);
    return 1;
  }
  if (n == 0) {
    printf("No spikes fired (empty file or too small k)\n");
  } else {
    for (long i = 0; i < n; ++i)
      printf("%3ld: Neuron %6llu \xe2\x86\x92 %8llu spikes (%u unique k-mers colliding)\n", i + 1,
             (unsigned long long)top[i].idx, (unsigned long long)top[i].spikes, top[i].uniques);
  }
  fprintf(stderr, "[INFO neurokmer] Processing complete - total spikes: %llu, energy: %s\n",
          (unsigned long long)nk_total_spikes(c), rust_f64(nk_energy_used(c)).c_str());
  printf("\nTotal spikes fired: %llu\n", (unsigned long long)nk_total_spikes(c));
  printf("Simulated energy used: %s\n", rust_f64(nk_energy_used(c)).c_str());
  printf("Neuron pool size used: %llu\n", pool);
  printf("Streaming mode: %s\n", streaming ? "true" : "false");
  nk_free(c);
  return 0;
}
