// host_asan_main.cpp -- drives the HIP-free host code of the drop-in (ont-tcrconsensus_amd/csrc/host_io.cpp)
// under AddressSanitizer + UndefinedBehaviorSanitizer for the CPU suite (tests/test_sanitizers_cpu.py), the way
// oracle/asan_main.c drives the oracle.  Test infrastructure: the product links host_io.cpp, never this file.
//
//   host_asan fasta <in.fa> <out.tsv>          read_fasta: "label\tsequence" per record
//   host_asan fastq <in.fq> <out.tsv>          read_fastq: the same
//   host_asan parse|parse_pre <in.fa> <sizes> <work_dir> <min> <max> <balance> <max_clusters>
//        parse_clusters over clusters of consecutive records (sizes: comma-separated cluster sizes); prints
//        "n_written reads_found reads_written empty_region" or "error <code> <message>"
//   host_asan write <in.fa> <sizes> <prefix> <consout>   write_consout (consensus = the centroid's sequence)
//        + write_cluster_files (masked = the sequences, cut at 128); write_input: the same from the input bytes
//   host_asan umis <in.fa> <res.txt> <out.fa> <a3>  write_detected_umis (res: 6 ints per record)
//   host_asan bgzf <in.bgzf> <out.raw>         inflate_bgzf
//   host_asan argv <args...>                   umiclust_params_from_argv: the decoded fields
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../ont-tcrconsensus_amd/csrc/host_io.h"

using namespace uc::io;

static std::vector<int32_t> sizes_of(const char* s) {
  std::vector<int32_t> v;
  for (const char* p = s; *p;) {
    v.push_back((int32_t)strtol(p, const_cast<char**>(&p), 10));
    if (*p == ',') p++;
  }
  return v;
}

static int dump(const Fasta& f, const char* out) {
  FILE* fo = fopen(out, "w");
  if (!fo) return 2;
  for (size_t i = 0; i < f.hdr_off.size(); i++) {
    fwrite(f.data + f.hdr_off[i], 1, (size_t)f.hdr_len[i], fo);
    fputc('\t', fo);
    fwrite(f.seq.data() + f.seq_off[i], 1, (size_t)(f.seq_off[i + 1] - f.seq_off[i]), fo);
    fputc('\n', fo);
  }
  fclose(fo);
  return 0;
}

struct Clusters {
  std::vector<int32_t> ostart, omemb, perm;
  ClusterView cv;
};

static bool clusters_of(const Fasta& f, const char* sizes, Clusters& C) {
  const std::vector<int32_t> sz = sizes_of(sizes);
  C.ostart.assign(1, 0);
  for (int32_t s : sz) C.ostart.push_back(C.ostart.back() + s);
  const int32_t n = (int32_t)f.hdr_off.size();
  if (C.ostart.back() != n) return false;
  C.omemb.resize((size_t)n);
  C.perm.resize((size_t)n);
  for (int32_t i = 0; i < n; i++) C.omemb[i] = C.perm[i] = i;
  C.cv = ClusterView{(int32_t)sz.size(), C.ostart.data(), C.omemb.data(), C.perm.data()};
  return true;
}

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  const std::string cmd = argv[1];
  try {
    if ((cmd == "fasta" || cmd == "fastq") && argc == 4) {
      Fasta f;
      if (!(cmd == "fasta" ? read_fasta(argv[2], f) : read_fastq(argv[2], f))) {
        printf("error read\n");
        return 0;
      }
      return dump(f, argv[3]);
    }
    if ((cmd == "parse" || cmd == "parse_pre") && argc == 9) {
      Fasta f;
      if (!read_fasta(argv[2], f)) return 3;
      Clusters C;
      if (!clusters_of(f, argv[3], C)) return 4;
      umiclust_parse_params pp{atoi(argv[5]), atoi(argv[6]), atoi(argv[7]), atoi(argv[8])};
      umiclust_parse_result pr{};
      try {
        std::vector<RecFields> pre;  // parse_pre: the header fields computed ahead, as the fused drop-in does
        if (cmd == "parse_pre") precompute_fields(f, pre, 3);
        parse_clusters(f, C.cv, &pp, argv[4], &pr, pre.empty() ? nullptr : pre.data());
        printf("%lld %lld %lld %d\n", (long long)pr.n_written, (long long)pr.reads_found, (long long)pr.reads_written,
               pr.empty_region);
      } catch (const IoError& e) {
        printf("error %d %s\n", e.code, e.msg.c_str());
      }
      return 0;
    }
    if ((cmd == "write" || cmd == "write_input") && argc == 6) {
      Fasta f;
      if (!read_fasta(argv[2], f)) return 3;
      Clusters C;
      if (!clusters_of(f, argv[3], C)) return 4;
      const int32_t K = C.cv.K, n = (int32_t)f.hdr_off.size();
      std::vector<char> cons;
      std::vector<int64_t> cons_off(1, 0);
      for (int32_t k = 0; k < K; k++) {
        const int32_t c = C.ostart[k];
        cons.insert(cons.end(), f.seq.begin() + f.seq_off[c], f.seq.begin() + f.seq_off[c + 1]);
        cons_off.push_back((int64_t)cons.size());
      }
      const int stride = 128;
      std::vector<char> masked((size_t)n * stride, 'N');
      std::vector<uint8_t> hlen((size_t)n);
      for (int32_t i = 0; i < n; i++) {
        const int64_t L = std::min<int64_t>(stride, f.seq_off[i + 1] - f.seq_off[i]);
        memcpy(masked.data() + (size_t)i * stride, f.seq.data() + f.seq_off[i], (size_t)L);
        hlen[i] = (uint8_t)L;
      }
      write_consout(argv[5], f, C.cv, cons.data(), cons_off.data(), true, 80);
      // write_input: no masked copy (no sequence changed): the input bytes, whole
      write_cluster_files(argv[4], f, C.cv, cmd == "write" ? masked.data() : nullptr, stride, hlen.data(), 80);
      return 0;
    }
    if (cmd == "umis" && argc == 6) {
      Fasta f;
      if (!read_fasta(argv[2], f)) return 3;
      std::vector<int32_t> res;
      FILE* fr = fopen(argv[3], "r");
      if (!fr) return 3;
      int v;
      while (fscanf(fr, "%d", &v) == 1) res.push_back(v);
      fclose(fr);
      const int64_t n = (int64_t)f.hdr_off.size();
      if ((int64_t)res.size() != 6 * n) return 4;
      printf("%lld\n", (long long)write_detected_umis(argv[4], f, res.data(), n, atoi(argv[5])));
      return 0;
    }
    if (cmd == "bgzf" && argc == 4) {
      std::vector<uint8_t> raw;
      if (!inflate_bgzf(argv[2], raw)) {
        printf("error bgzf\n");
        return 0;
      }
      FILE* fo = fopen(argv[3], "wb");
      if (!fo) return 2;
      if (!raw.empty()) fwrite(raw.data(), 1, raw.size(), fo);
      fclose(fo);
      return 0;
    }
    if (cmd == "argv") {
      umiclust_params p;
      char in[256], cl[256], co[256], lg[256];
      const int rc = umiclust_params_from_argv(&p, argc - 2, (const char* const*)(argv + 2), in, cl, co, lg, 256);
      if (rc != UMICLUST_OK) {
        printf("rc %d\n", rc);
        return 0;
      }
      printf("id %.4f len %d %d match %d mismatch %d open", p.id, p.minseqlength, p.maxseqlength, p.match, p.mismatch);
      for (int k = 0; k < 6; k++) printf(" %d", p.gap_open[k]);
      printf(" ext");
      for (int k = 0; k < 6; k++) printf(" %d", p.gap_ext[k]);
      printf(" strand %d sort %d id %d threads %d o4 %d in %s clusters %s consout %s log %s\n", p.strand_both,
             p.clusterout_sort, p.clusterout_id, p.threads, p.policy_threads, in, cl, co, lg);
      return 0;
    }
  } catch (const IoError& e) {
    printf("error %d %s\n", e.code, e.msg.c_str());
    return 0;
  }
  return 2;
}
