#include "scheduler.h"

#include <algorithm>
#include <cmath>
#include <limits>
#include <set>

namespace caamd_rt {

static constexpr double kEps = 1e-9;

int ClusterScheduler::rid(const std::string& name) {
  auto it = res_ids_.find(name);
  if (it != res_ids_.end()) return it->second;
  const int id = (int)res_names_.size();
  res_ids_[name] = id;
  res_names_.push_back(name);
  for (auto& n : nodes_) {
    n.total.resize(res_names_.size(), 0.0);
    n.avail.resize(res_names_.size(), 0.0);
  }
  return id;
}

int ClusterScheduler::rid_const(const std::string& name) const {
  auto it = res_ids_.find(name);
  return it == res_ids_.end() ? -1 : it->second;
}

std::vector<std::pair<int, double>> ClusterScheduler::to_vec(const ResMap& m) {
  std::vector<std::pair<int, double>> v;
  for (auto& kv : m)
    if (kv.second > 0) v.emplace_back(rid(kv.first), kv.second);
  return v;
}

void ClusterScheduler::add_node(const std::string& id, const ResMap& total) {
  if (node_idx_.count(id)) remove_node(id);
  NodeRes n;
  n.id = id;
  n.total.assign(res_names_.size(), 0.0);
  n.avail.assign(res_names_.size(), 0.0);
  node_idx_[id] = (int)nodes_.size();
  nodes_.push_back(n);
  for (auto& kv : total) {
    const int r = rid(kv.first);
    nodes_[node_idx_[id]].total[r] = kv.second;
    nodes_[node_idx_[id]].avail[r] = kv.second;
  }
}

void ClusterScheduler::remove_node(const std::string& id) {
  auto it = node_idx_.find(id);
  if (it == node_idx_.end()) return;
  const int i = it->second;
  nodes_.erase(nodes_.begin() + i);
  node_idx_.clear();
  for (int j = 0; j < (int)nodes_.size(); ++j) node_idx_[nodes_[j].id] = j;
}

void ClusterScheduler::set_alive(const std::string& id, bool alive) {
  auto it = node_idx_.find(id);
  if (it != node_idx_.end()) nodes_[it->second].alive = alive;
}

ResMap ClusterScheduler::total(const std::string& id) const {
  ResMap m;
  auto it = node_idx_.find(id);
  if (it == node_idx_.end()) return m;
  const auto& n = nodes_[it->second];
  for (size_t r = 0; r < res_names_.size(); ++r)
    if (n.total[r] > kEps) m[res_names_[r]] = n.total[r];
  return m;
}

ResMap ClusterScheduler::available(const std::string& id) const {
  ResMap m;
  auto it = node_idx_.find(id);
  if (it == node_idx_.end()) return m;
  const auto& n = nodes_[it->second];
  for (size_t r = 0; r < res_names_.size(); ++r)
    if (n.total[r] > kEps) m[res_names_[r]] = std::max(0.0, n.avail[r]);
  return m;
}

ResMap ClusterScheduler::cluster_total() const {
  ResMap m;
  for (auto& n : nodes_)
    if (n.alive)
      for (size_t r = 0; r < res_names_.size(); ++r)
        if (n.total[r] > kEps) m[res_names_[r]] += n.total[r];
  return m;
}

ResMap ClusterScheduler::cluster_available() const {
  ResMap m;
  for (auto& n : nodes_)
    if (n.alive)
      for (size_t r = 0; r < res_names_.size(); ++r)
        if (n.total[r] > kEps) m[res_names_[r]] += std::max(0.0, n.avail[r]);
  return m;
}

std::vector<std::string> ClusterScheduler::nodes() const {
  std::vector<std::string> v;
  for (auto& n : nodes_) v.push_back(n.id);
  return v;
}

bool ClusterScheduler::fits(const NodeRes& n, const std::vector<std::pair<int, double>>& d,
                            bool use_total) const {
  for (auto& kv : d) {
    const double have = use_total ? n.total[kv.first] : n.avail[kv.first];
    if (have + kEps < kv.second) return false;
  }
  return true;
}

double ClusterScheduler::utilization(const NodeRes& n) const {
  // max utilisation over the node's real (non-group) resources
  double u = 0.0;
  for (size_t r = 0; r < res_names_.size(); ++r) {
    if (n.total[r] <= kEps || res_names_[r].find("_group_") != std::string::npos) continue;
    u = std::max(u, 1.0 - n.avail[r] / n.total[r]);
  }
  return u;
}

void ClusterScheduler::set_labels(const std::string& id, const LabelMap& labels) {
  auto it = node_idx_.find(id);
  if (it != node_idx_.end()) nodes_[it->second].labels = labels;
}

LabelMap ClusterScheduler::labels(const std::string& id) const {
  auto it = node_idx_.find(id);
  return it == node_idx_.end() ? LabelMap{} : nodes_[it->second].labels;
}

bool ClusterScheduler::labels_match(const LabelMap& labels, const std::vector<LabelCond>& conds) {
  for (const auto& c : conds) {
    auto it = labels.find(c.key);
    const bool has = it != labels.end();
    switch ((LabelOp)c.op) {
      case LabelOp::kIn:
        if (!has || std::find(c.values.begin(), c.values.end(), it->second) == c.values.end())
          return false;
        break;
      case LabelOp::kNotIn:
        if (has && std::find(c.values.begin(), c.values.end(), it->second) != c.values.end())
          return false;
        break;
      case LabelOp::kExists:
        if (!has) return false;
        break;
      case LabelOp::kDoesNotExist:
        if (has) return false;
        break;
    }
  }
  return true;
}

std::string ClusterScheduler::pick_node(const ResMap& demand, int strategy,
                                        const std::string& affinity_node, bool soft,
                                        const std::string& preferred_node,
                                        const std::vector<LabelCond>& hard,
                                        const std::vector<LabelCond>& soft_labels) {
  const auto d = to_vec(demand);
  bool feasible_any = false;
  for (auto& n : nodes_)
    if (n.alive && fits(n, d, true) && labels_match(n.labels, hard)) feasible_any = true;
  if (!feasible_any) return "!";
  if ((Strategy)strategy == Strategy::kLabel) {
    // hard conditions filter; among the matching nodes prefer those that also meet
    // the soft conditions, then the least utilised one
    int best = -1, best_soft = -1;
    double best_u = std::numeric_limits<double>::max();
    for (int i = 0; i < (int)nodes_.size(); ++i) {
      auto& n = nodes_[i];
      if (!n.alive || !labels_match(n.labels, hard) || !fits(n, d, false)) continue;
      const int s = soft_labels.empty() ? 0 : (labels_match(n.labels, soft_labels) ? 1 : 0);
      const double u = utilization(n);
      if (s > best_soft || (s == best_soft && u < best_u)) {
        best = i;
        best_soft = s;
        best_u = u;
      }
    }
    return best < 0 ? "" : nodes_[best].id;
  }
  if ((Strategy)strategy == Strategy::kNodeAffinity) {
    auto it = node_idx_.find(affinity_node);
    if (it != node_idx_.end() && nodes_[it->second].alive) {
      auto& n = nodes_[it->second];
      if (fits(n, d, false)) return n.id;
      if (!soft) return fits(n, d, true) ? "" : "!";
    } else if (!soft) {
      return "!";
    }
    // soft: fall through to the default policy
  }
  if ((Strategy)strategy == Strategy::kSpread) {
    // round robin over feasible nodes, least utilised first on ties
    const size_t N = nodes_.size();
    for (size_t k = 0; k < N; ++k) {
      auto& n = nodes_[(rr_ + k) % N];
      if (n.alive && fits(n, d, false)) {
        rr_ = (rr_ + k + 1) % N;
        return n.id;
      }
    }
    return "";
  }
  // hybrid: preferred (local) node while below the spread threshold, then the
  // least-utilised feasible node
  auto pit = node_idx_.find(preferred_node);
  if (pit != node_idx_.end()) {
    auto& n = nodes_[pit->second];
    if (n.alive && fits(n, d, false) && utilization(n) < spread_threshold_) return n.id;
  }
  int best = -1;
  double best_u = std::numeric_limits<double>::max();
  for (int i = 0; i < (int)nodes_.size(); ++i) {
    auto& n = nodes_[i];
    if (!n.alive || !fits(n, d, false)) continue;
    const double u = utilization(n);
    if (u < best_u) {
      best_u = u;
      best = i;
    }
  }
  return best < 0 ? "" : nodes_[best].id;
}

bool ClusterScheduler::acquire(const std::string& node, const ResMap& demand) {
  auto it = node_idx_.find(node);
  if (it == node_idx_.end()) return false;
  auto& n = nodes_[it->second];
  const auto d = to_vec(demand);
  if (!fits(n, d, false)) return false;
  for (auto& kv : d) n.avail[kv.first] -= kv.second;
  return true;
}

void ClusterScheduler::release(const std::string& node, const ResMap& demand) {
  auto it = node_idx_.find(node);
  if (it == node_idx_.end()) return;
  auto& n = nodes_[it->second];
  for (auto& kv : demand) {
    const int r = rid(kv.first);
    n.avail[r] = std::min(n.total[r], n.avail[r] + kv.second);
  }
}

std::vector<std::string> ClusterScheduler::place_bundles(const std::vector<ResMap>& bundles,
                                                         int strategy, bool use_total) {
  std::vector<std::vector<std::pair<int, double>>> bv;
  for (auto& b : bundles) bv.push_back(to_vec(b));
  std::vector<std::vector<double>> avail;  // simulated availability
  for (auto& n : nodes_) avail.push_back(use_total ? n.total : n.avail);
  auto fits_sim = [&](int ni, const std::vector<std::pair<int, double>>& d) {
    if (!nodes_[ni].alive) return false;
    for (auto& kv : d)
      if (avail[ni][kv.first] + kEps < kv.second) return false;
    return true;
  };
  auto take = [&](int ni, const std::vector<std::pair<int, double>>& d) {
    for (auto& kv : d) avail[ni][kv.first] -= kv.second;
  };
  std::vector<std::string> out(bundles.size());
  const int N = (int)nodes_.size();
  switch ((PgStrategy)strategy) {
    case PgStrategy::kStrictPack: {
      for (int ni = 0; ni < N; ++ni) {
        auto saved = avail[ni];
        bool ok = true;
        for (auto& d : bv) {
          if (!fits_sim(ni, d)) {
            ok = false;
            break;
          }
          take(ni, d);
        }
        if (ok) {
          for (auto& o : out) o = nodes_[ni].id;
          return out;
        }
        avail[ni] = saved;
      }
      return {};
    }
    case PgStrategy::kStrictSpread: {
      std::set<int> used;
      for (size_t b = 0; b < bv.size(); ++b) {
        int pick = -1;
        for (int ni = 0; ni < N; ++ni)
          if (!used.count(ni) && fits_sim(ni, bv[b])) {
            pick = ni;
            break;
          }
        if (pick < 0) return {};
        used.insert(pick);
        take(pick, bv[b]);
        out[b] = nodes_[pick].id;
      }
      return out;
    }
    case PgStrategy::kSpread: {
      int start = 0;
      for (size_t b = 0; b < bv.size(); ++b) {
        int pick = -1;
        for (int k = 0; k < N; ++k) {
          const int ni = (start + k) % N;
          if (fits_sim(ni, bv[b])) {
            pick = ni;
            break;
          }
        }
        if (pick < 0) return {};
        take(pick, bv[b]);
        out[b] = nodes_[pick].id;
        start = pick + 1;
      }
      return out;
    }
    case PgStrategy::kPack:
    default: {
      for (size_t b = 0; b < bv.size(); ++b) {
        int pick = -1;
        // prefer the node already used by the previous bundle
        if (b > 0) {
          const int prev = node_idx_[out[b - 1]];
          if (fits_sim(prev, bv[b])) pick = prev;
        }
        for (int ni = 0; pick < 0 && ni < N; ++ni)
          if (fits_sim(ni, bv[b])) pick = ni;
        if (pick < 0) return {};
        take(pick, bv[b]);
        out[b] = nodes_[pick].id;
      }
      return out;
    }
  }
}

bool ClusterScheduler::pg_feasible(const std::vector<ResMap>& bundles, int strategy) const {
  return !const_cast<ClusterScheduler*>(this)->place_bundles(bundles, strategy, true).empty() ||
         bundles.empty();
}

std::vector<std::string> ClusterScheduler::reserve_pg(const std::string& pg_id,
                                                      const std::vector<ResMap>& bundles,
                                                      int strategy) {
  auto placement = place_bundles(bundles, strategy, false);
  if (placement.empty() && !bundles.empty()) return {};
  for (size_t b = 0; b < bundles.size(); ++b) {
    auto& node = nodes_[node_idx_[placement[b]]];
    for (auto& kv : bundles[b]) {
      if (kv.second <= 0) continue;
      node.avail[rid(kv.first)] -= kv.second;
      const int gi = rid(kv.first + "_group_" + std::to_string(b) + "_" + pg_id);
      const int ga = rid(kv.first + "_group_" + pg_id);
      auto& n2 = nodes_[node_idx_[placement[b]]];  // rid() may have resized vectors
      n2.total[gi] += kv.second;
      n2.avail[gi] += kv.second;
      n2.total[ga] += kv.second;
      n2.avail[ga] += kv.second;
    }
    // the "bundle" marker resource lets an empty-demand task target a bundle
    const int bi = rid("bundle_group_" + std::to_string(b) + "_" + pg_id);
    const int ba = rid("bundle_group_" + pg_id);
    auto& n3 = nodes_[node_idx_[placement[b]]];
    n3.total[bi] += 1000;
    n3.avail[bi] += 1000;
    n3.total[ba] += 1000;
    n3.avail[ba] += 1000;
  }
  pgs_[pg_id] = PgRecord{placement, bundles};
  return placement;
}

void ClusterScheduler::remove_pg(const std::string& pg_id) {
  auto it = pgs_.find(pg_id);
  if (it == pgs_.end()) return;
  const std::string suffix = "_group_";
  for (size_t b = 0; b < it->second.bundles.size(); ++b) {
    auto nit = node_idx_.find(it->second.nodes[b]);
    if (nit == node_idx_.end()) continue;
    auto& node = nodes_[nit->second];
    for (auto& kv : it->second.bundles[b]) {
      if (kv.second <= 0) continue;
      const int r = rid(kv.first);
      node.avail[r] = std::min(node.total[r], node.avail[r] + kv.second);
    }
  }
  // zero every virtual resource of this group
  const std::string tag = "_" + pg_id;
  for (size_t r = 0; r < res_names_.size(); ++r) {
    const auto& nm = res_names_[r];
    if (nm.size() > tag.size() && nm.compare(nm.size() - tag.size(), tag.size(), tag) == 0 &&
        nm.find(suffix) != std::string::npos)
      for (auto& n : nodes_) n.total[r] = n.avail[r] = 0.0;
  }
  pgs_.erase(it);
}

}  // namespace caamd_rt
