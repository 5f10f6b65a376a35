// cg_jobset.h -- the interned job model behind cg_jobset_* (cg_jobset.cpp)
// and the bulk JSON ingestion (cg_ingest.cpp).
#pragma once
#include <algorithm>
#include <string>
#include <unordered_map>
#include <vector>

#include "../../include/cronsun_gpu.h"

int cg_fail(int code, const std::string& msg);

struct cg_jobset {
  std::unordered_map<std::string, int32_t> node_idx, group_idx;
  std::vector<std::string> node_ids, group_ids;
  std::vector<std::vector<int32_t>> group_nodes;
  std::vector<uint8_t> group_exists;
  std::vector<std::string> job_ids;
  std::vector<uint8_t> job_pause;
  std::vector<int32_t> job_first_rule;
  std::vector<std::string> rule_ids;
  std::vector<int32_t> rule_job;
  std::vector<std::vector<int32_t>> r_nids, r_gids, r_ex;
  // filled by the JSON ingestion (cg_ingest.cpp); defaults for add_job/add_rule
  std::vector<int32_t> job_kind;        // Job.Kind
  std::vector<int64_t> job_avg;         // Job.AvgTime (ms)
  std::vector<int64_t> job_parallels;   // Job.Parallels after alone()
  std::vector<cg_schedule> rule_sched;  // JobRule.Schedule (JobRule.Valid)
  std::vector<uint8_t> rule_has_sched;
  // frozen arrays
  std::vector<int64_t> f_group_off, f_nid_off, f_gid_off, f_ex_off;
  std::vector<int32_t> f_group_nodes, f_nids, f_gids, f_ex;
  std::vector<int32_t> f_rule_key;  // interned Rule.ID (Cmd key within a job)

  int32_t node(const std::string& id) {
    auto it = node_idx.find(id);
    if (it != node_idx.end()) return it->second;
    int32_t k = int32_t(node_ids.size());
    node_ids.push_back(id);
    node_idx.emplace(id, k);
    return k;
  }
  int32_t group(const std::string& id) {
    auto it = group_idx.find(id);
    if (it != group_idx.end()) return it->second;
    int32_t k = int32_t(group_ids.size());
    group_ids.push_back(id);
    group_idx.emplace(id, k);
    group_nodes.emplace_back();
    group_exists.push_back(0);
    return k;
  }
  int32_t node(const char* id) {
    auto it = node_idx.find(id);
    if (it != node_idx.end()) return it->second;
    int32_t k = int32_t(node_ids.size());
    node_ids.emplace_back(id);
    node_idx.emplace(node_ids.back(), k);
    return k;
  }
  int32_t group(const char* id) {
    auto it = group_idx.find(id);
    if (it != group_idx.end()) return it->second;
    int32_t k = int32_t(group_ids.size());
    group_ids.emplace_back(id);
    group_idx.emplace(group_ids.back(), k);
    group_nodes.emplace_back();
    group_exists.push_back(0);
    return k;
  }
  int32_t find_node(const char* id) const {
    auto it = node_idx.find(id);
    return it == node_idx.end() ? -1 : it->second;
  }
  bool in_list(const std::vector<int32_t>& v, int32_t x) const {
    return std::find(v.begin(), v.end(), x) != v.end();
  }
  // JobRule.included + Group.Included
  bool included(int32_t r, int32_t n) const {
    if (n < 0) return false;
    if (in_list(r_nids[r], n)) return true;
    for (int32_t g : r_gids[r])
      if (group_exists[g] && in_list(group_nodes[g], n)) return true;
    return false;
  }
  int32_t rule_end(int32_t job) const {
    return job + 1 < int32_t(job_first_rule.size()) ? job_first_rule[job + 1]
                                                     : int32_t(rule_ids.size());
  }
};

