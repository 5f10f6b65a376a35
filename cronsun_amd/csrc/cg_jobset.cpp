// cg_jobset.cpp -- cronsun's string-keyed Job/JobRule/Group model interned
// into the integer arrays of cg_rules_in, plus the reference's per-node
// resolution functions on the host:
//   Job.Cmds     job.go:591-614   (Pause => none; ExcludeNodeIDs is a no-op
//                                  because its `continue` binds to the inner
//                                  loop, job.go:598-602; map keyed by
//                                  Job.ID + Rule.ID, later rules overwrite)
//   Job.IsRunOn  job.go:616-630   (ignores Pause)
//   JobRule.included job.go:274-288, Group.Included group.go:111-119
//   Job.GetJobNodes web/job.go:222-257 (cumulative excludes, first-seen order)
#include <cstring>
#include <map>

#include "cg_jobset.h"

extern "C" {

int cg_jobset_new(cg_jobset** out) {
  if (!out) return cg_fail(CG_EINVAL, "cg_jobset_new: null");
  *out = new cg_jobset();
  return CG_OK;
}

void cg_jobset_free(cg_jobset* js) { delete js; }

int cg_jobset_add_group(cg_jobset* js, const char* gid, const char* const* nids, size_t n) {
  if (!js || !gid || (n && !nids)) return cg_fail(CG_EINVAL, "cg_jobset_add_group: null");
  int32_t g = js->group(gid);
  js->group_exists[g] = 1;
  js->group_nodes[g].clear();  // groups map: the last definition of a gid wins
  for (size_t i = 0; i < n; i++) js->group_nodes[g].push_back(js->node(nids[i]));
  return CG_OK;
}

int cg_jobset_add_job(cg_jobset* js, const char* job_id, int pause) {
  if (!js || !job_id) return cg_fail(CG_EINVAL, "cg_jobset_add_job: null");
  js->job_ids.emplace_back(job_id);
  js->job_pause.push_back(pause ? 1 : 0);
  js->job_first_rule.push_back(int32_t(js->rule_ids.size()));
  js->job_kind.push_back(0);
  js->job_avg.push_back(0);
  js->job_parallels.push_back(0);
  return CG_OK;
}

int cg_jobset_add_rule(cg_jobset* js, const char* rule_id, const char* const* gids, size_t ng,
                       const char* const* nids, size_t nn, const char* const* ex, size_t ne) {
  if (!js || !rule_id || (ng && !gids) || (nn && !nids) || (ne && !ex))
    return cg_fail(CG_EINVAL, "cg_jobset_add_rule: null");
  if (js->job_ids.empty()) return cg_fail(CG_EINVAL, "cg_jobset_add_rule: no job added yet");
  js->rule_ids.emplace_back(rule_id);
  js->rule_job.push_back(int32_t(js->job_ids.size()) - 1);
  std::vector<int32_t> a, b, c;
  for (size_t i = 0; i < ng; i++) a.push_back(js->group(gids[i]));
  for (size_t i = 0; i < nn; i++) b.push_back(js->node(nids[i]));
  for (size_t i = 0; i < ne; i++) c.push_back(js->node(ex[i]));
  js->r_gids.push_back(std::move(a));
  js->r_nids.push_back(std::move(b));
  js->r_ex.push_back(std::move(c));
  js->rule_sched.push_back(cg_schedule{});
  js->rule_has_sched.push_back(0);
  return CG_OK;
}

int cg_jobset_rules(cg_jobset* js, cg_rules_in* out) {
  if (!js || !out) return cg_fail(CG_EINVAL, "cg_jobset_rules: null");
  auto flatten = [](const std::vector<std::vector<int32_t>>& v, std::vector<int64_t>& off,
                    std::vector<int32_t>& flat) {
    off.assign(1, 0);
    flat.clear();
    for (auto& x : v) {
      flat.insert(flat.end(), x.begin(), x.end());
      off.push_back(int64_t(flat.size()));
    }
  };
  flatten(js->group_nodes, js->f_group_off, js->f_group_nodes);
  flatten(js->r_nids, js->f_nid_off, js->f_nids);
  flatten(js->r_gids, js->f_gid_off, js->f_gids);
  flatten(js->r_ex, js->f_ex_off, js->f_ex);
  out->n_nodes = int32_t(js->node_ids.size());
  out->n_groups = int32_t(js->group_ids.size());
  out->n_rules = int32_t(js->rule_ids.size());
  out->n_jobs = int32_t(js->job_ids.size());
  out->group_off = js->f_group_off.data();
  out->group_nodes = js->f_group_nodes.data();
  out->group_exists = js->group_exists.data();
  out->rule_job = js->rule_job.data();
  out->nid_off = js->f_nid_off.data();
  out->nids = js->f_nids.data();
  out->gid_off = js->f_gid_off.data();
  out->gids = js->f_gids.data();
  out->ex_off = js->f_ex_off.data();
  out->ex = js->f_ex.data();
  out->job_pause = js->job_pause.data();
  // Cmd.GetID() = Job.ID + Rule.ID (job.go:130-132): within one job two keys
  // are equal exactly when the Rule.IDs are, so interning the Rule.IDs is
  // enough (raw IDs: the node path never trims them, only Job.Check does)
  std::unordered_map<std::string, int32_t> key_idx;
  js->f_rule_key.resize(js->rule_ids.size());
  for (size_t r = 0; r < js->rule_ids.size(); r++)
    js->f_rule_key[r] = key_idx.emplace(js->rule_ids[r], int32_t(key_idx.size())).first->second;
  out->rule_key = js->f_rule_key.empty() ? nullptr : js->f_rule_key.data();
  return CG_OK;
}

int32_t cg_jobset_node_index(const cg_jobset* js, const char* nid) {
  if (!js || !nid) return -1;
  return js->find_node(nid);
}

const char* cg_jobset_node_id(const cg_jobset* js, int32_t idx) {
  if (!js || idx < 0 || idx >= int32_t(js->node_ids.size())) return nullptr;
  return js->node_ids[idx].c_str();
}

int32_t cg_jobset_cmds(const cg_jobset* js, int32_t job, const char* nid, int32_t* rules_out,
                       int32_t cap) {
  if (!js || !nid || job < 0 || job >= int32_t(js->job_ids.size()))
    return cg_fail(CG_EINVAL, "cg_jobset_cmds: bad argument");
  if (js->job_pause[job]) return 0;  // job.go:593
  const int32_t n = js->find_node(nid);
  std::map<std::string, int32_t> cmds;  // Cmd.GetID() -> rule (later rules overwrite)
  for (int32_t r = js->job_first_rule[job]; r < js->rule_end(job); r++) {
    // the ExcludeNodeIDs loop of job.go:598-602 has no effect
    if (js->included(r, n)) cmds[js->job_ids[job] + js->rule_ids[r]] = r;
  }
  std::vector<int32_t> rs;
  for (auto& kv : cmds) rs.push_back(kv.second);
  std::sort(rs.begin(), rs.end());
  int32_t k = 0;
  for (int32_t r : rs) {
    if (rules_out && k < cap) rules_out[k] = r;
    k++;
  }
  return k;
}

int cg_jobset_is_run_on(const cg_jobset* js, int32_t job, const char* nid) {
  if (!js || !nid || job < 0 || job >= int32_t(js->job_ids.size()))
    return cg_fail(CG_EINVAL, "cg_jobset_is_run_on: bad argument");
  const int32_t n = js->find_node(nid);
  for (int32_t r = js->job_first_rule[job]; r < js->rule_end(job); r++)
    if (js->included(r, n)) return 1;
  return 0;
}

int32_t cg_jobset_job_nodes(const cg_jobset* js, int32_t job, int32_t* nodes_out, int32_t cap) {
  if (!js || job < 0 || job >= int32_t(js->job_ids.size()))
    return cg_fail(CG_EINVAL, "cg_jobset_job_nodes: bad argument");
  std::vector<int32_t> nodes, ex;
  for (int32_t r = js->job_first_rule[job]; r < js->rule_end(job); r++) {
    std::vector<int32_t> in = nodes;  // append(nodes, rule.NodeIDs...)
    in.insert(in.end(), js->r_nids[r].begin(), js->r_nids[r].end());
    for (int32_t g : js->r_gids[r])
      if (js->group_exists[g])
        in.insert(in.end(), js->group_nodes[g].begin(), js->group_nodes[g].end());
    ex.insert(ex.end(), js->r_ex[r].begin(), js->r_ex[r].end());
    for (int32_t x : in)  // SubtractStringArray(inNodes, exNodes)
      if (!js->in_list(ex, x)) nodes.push_back(x);
  }
  std::vector<int32_t> uniq;  // UniqueStringArray: first-seen order
  for (int32_t x : nodes)
    if (!js->in_list(uniq, x)) uniq.push_back(x);
  int32_t k = 0;
  for (int32_t x : uniq) {
    if (nodes_out && k < cap) nodes_out[k] = x;
    k++;
  }
  return k;
}

}  // extern "C"
