// Host parsers of the library under AddressSanitizer + UndefinedBehavior-
// Sanitizer: the etcd JSON decoder (cg_ingest.cpp), job interning
// (cg_jobset.cpp), the spec parser (cg_parse.cpp) and the TZif reader / plan
// builder (cg_zone.cpp) -- every input that reaches the library from outside.
// Test infrastructure: tests/test_sanitizers.py builds this with
// -fsanitize=address,undefined and feeds it hostile inputs.
//
// Input file: records of {u32 kind, u32 len, len bytes}; kind 0 = group JSON,
// 1 = job JSON, 2 = spec string, 3 = TZif blob, 4 = duration string, 5 = field
// expression.
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../cronsun_amd/csrc/cg_jobset.h"
#include "../../cronsun_amd/csrc/cg_parse.h"
#include "../../cronsun_amd/csrc/cg_zone.h"
#include "../../include/cronsun_gpu.h"

// the library's error sink lives in cg_api.cpp (HIP); a plain one here
int cg_fail(int code, const std::string& msg) {
  (void)msg;
  return code;
}

using namespace cg;

int main(int argc, char** argv) {
  if (argc < 2) return 2;
  FILE* f = fopen(argv[1], "rb");
  if (!f) return 2;
  std::vector<std::string> rec[6];
  for (;;) {
    uint32_t hdr[2];
    if (fread(hdr, 4, 2, f) != 2) break;
    std::string b(hdr[1], '\0');
    if (hdr[1] && fread(&b[0], 1, hdr[1], f) != hdr[1]) break;
    if (hdr[0] < 6) rec[hdr[0]].push_back(std::move(b));
  }
  fclose(f);
  long ok[6] = {0, 0, 0, 0, 0, 0};

  // etcd values -> jobset (GetGroups / GetJobs batch form), then every reader
  {
    cg_jobset* js = nullptr;
    if (cg_jobset_new(&js) != CG_OK) return 3;
    for (int kind = 0; kind < 2; kind++) {
      std::vector<const char*> docs;
      std::vector<size_t> lens;
      for (auto& d : rec[kind]) {
        docs.push_back(d.data());
        lens.push_back(d.size());
      }
      std::vector<int32_t> st(docs.size() + 1, -1);
      int rc = kind == 0 ? cg_jobset_ingest_groups(js, docs.data(), lens.data(), docs.size(), 4, st.data())
                         : cg_jobset_ingest_jobs(js, docs.data(), lens.data(), docs.size(), 4, st.data());
      if (rc != CG_OK) return 4;
      for (size_t i = 0; i < docs.size(); i++) ok[kind] += st[i] == CG_INGEST_OK;
    }
    cg_rules_in rin;
    if (cg_jobset_rules(js, &rin) != CG_OK) return 5;
    std::vector<cg_schedule> sch(size_t(rin.n_rules) + 1);
    cg_jobset_schedules(js, sch.data(), sch.size());
    std::vector<int32_t> kind(size_t(rin.n_jobs) + 1);
    std::vector<int64_t> avg(size_t(rin.n_jobs) + 1), par(size_t(rin.n_jobs) + 1);
    cg_jobset_job_meta(js, kind.data(), avg.data(), par.data(), kind.size());
    std::vector<int32_t> out(size_t(rin.n_rules + rin.n_nodes) + 1);
    for (int32_t j = 0; j < rin.n_jobs; j++) {
      (void)cg_jobset_job_id(js, j);
      cg_jobset_job_nodes(js, j, out.data(), int32_t(out.size()));
      for (int32_t n = 0; n < rin.n_nodes && n < 8; n++) {
        const char* nid = cg_jobset_node_id(js, n);
        cg_jobset_cmds(js, j, nid, out.data(), int32_t(out.size()));
        cg_jobset_is_run_on(js, j, nid);
      }
      cg_jobset_cmds(js, j, "no-such-node", out.data(), int32_t(out.size()));
    }
    for (int32_t r = 0; r < rin.n_rules; r++) (void)cg_jobset_rule_id(js, r);
    for (int32_t g = 0; g < rin.n_groups; g++) (void)cg_jobset_group_id(js, g);
    cg_jobset_free(js);
  }

  // spec strings through every parser option set (parser.go:78-377)
  const int opts[] = {CG_PARSE_DEFAULT, CG_PARSE_STANDARD, 1 | 2 | 4 | 8 | 16 | 32,
                      2 | 4 | 8 | 16 | 64, 4 | 8 | 16 | 32 | 128, 128};
  for (auto& s : rec[2]) {
    for (int o : opts) {
      Schedule out;
      std::string err;
      ok[2] += parse(o, std::string_view(s), &out, &err) == 0;
    }
  }
  for (auto& s : rec[4]) {
    int64_t d;
    std::string err;
    ok[4] += parse_duration(std::string_view(s), &d, &err) == 0;
  }
  for (auto& s : rec[5]) {
    uint64_t bits;
    std::string err;
    for (int names = 0; names < 3; names++) {
      ok[5] += get_field(std::string_view(s), 0, 59, names, &bits, &err) == 0;
      get_range(std::string_view(s), 1, 31, names, &bits, &err);
    }
  }

  // TZif blobs (LoadLocationFromTZData), then the plan builder on what loads
  for (auto& b : rec[3]) {
    ZoneRules zr;
    std::string err;
    if (!zone_from_tzif(reinterpret_cast<const uint8_t*>(b.data()), b.size(), &zr, &err)) continue;
    ok[3]++;
    const int64_t probes[] = {INT64_MIN / 4, -62135596800LL, 0, 1767571200, 4102444800LL, 1LL << 40};
    for (int64_t t : probes) (void)zr.offset(t);
    ZoneTable t = build_table(zr, 1735689600, 1830297600);
    Plan p = build_plan(zr, 1767571200, 1767571200 + 400 * 86400);
    Plan q = build_plan(zr, -2208988800LL, -2208988800LL + 30 * 86400);
    (void)t;
    (void)p;
    (void)q;
  }
  printf("records groups=%zu jobs=%zu specs=%zu tzif=%zu durations=%zu fields=%zu\n", rec[0].size(),
         rec[1].size(), rec[2].size(), rec[3].size(), rec[4].size(), rec[5].size());
  printf("accepted groups=%ld jobs=%ld spec-parses=%ld tzif=%ld durations=%ld fields=%ld\n", ok[0], ok[1],
         ok[2], ok[3], ok[4], ok[5]);
  return 0;
}
