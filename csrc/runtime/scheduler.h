// Cluster resource scheduler (reference: src/ray/raylet/scheduling/
// cluster_resource_scheduler.cc + placement_group_resource_manager.cc).
// Holds total/available resource vectors per node, picks a node for a demand
// with the hybrid pack-then-spread policy, SPREAD or NODE_AFFINITY, and
// reserves placement-group bundles (PACK / SPREAD / STRICT_PACK /
// STRICT_SPREAD) by converting each bundle into per-bundle and per-group
// "virtual" resources on the chosen node (CPU -> CPU_group_<i>_<pg> and
// CPU_group_<pg>), which tasks scheduled into the group then consume.
#pragma once
#include <map>
#include <string>
#include <unordered_map>
#include <vector>

namespace caamd_rt {

using ResMap = std::map<std::string, double>;
using LabelMap = std::map<std::string, std::string>;

// One node-label condition (reference: python/ray/util/scheduling_strategies.py:135
// In / NotIn / Exists / DoesNotExist).
enum class LabelOp { kIn = 0, kNotIn = 1, kExists = 2, kDoesNotExist = 3 };
struct LabelCond {
  std::string key;
  int op;
  std::vector<std::string> values;
};

enum class Strategy { kHybrid = 0, kSpread = 1, kNodeAffinity = 2, kLabel = 3 };
enum class PgStrategy { kPack = 0, kSpread = 1, kStrictPack = 2, kStrictSpread = 3 };

struct NodeRes {
  std::string id;
  std::vector<double> total, avail;
  bool alive = true;
  LabelMap labels;
};

class ClusterScheduler {
 public:
  explicit ClusterScheduler(double spread_threshold = 0.5) : spread_threshold_(spread_threshold) {}

  void add_node(const std::string& id, const ResMap& total);
  void remove_node(const std::string& id);
  void set_alive(const std::string& id, bool alive);
  ResMap total(const std::string& id) const;
  ResMap available(const std::string& id) const;
  ResMap cluster_total() const;
  ResMap cluster_available() const;
  std::vector<std::string> nodes() const;

  // "" = not schedulable right now, "!" = infeasible on every node (even when idle)
  std::string pick_node(const ResMap& demand, int strategy, const std::string& affinity_node,
                        bool soft, const std::string& preferred_node,
                        const std::vector<LabelCond>& hard = {},
                        const std::vector<LabelCond>& soft_labels = {});
  void set_labels(const std::string& id, const LabelMap& labels);
  LabelMap labels(const std::string& id) const;
  static bool labels_match(const LabelMap& labels, const std::vector<LabelCond>& conds);
  bool acquire(const std::string& node, const ResMap& demand);
  void release(const std::string& node, const ResMap& demand);

  // returns node per bundle, or empty vector if it cannot be placed now
  std::vector<std::string> reserve_pg(const std::string& pg_id, const std::vector<ResMap>& bundles,
                                      int strategy);
  void remove_pg(const std::string& pg_id);
  bool pg_feasible(const std::vector<ResMap>& bundles, int strategy) const;

 private:
  int rid(const std::string& name);
  int rid_const(const std::string& name) const;
  bool fits(const NodeRes& n, const std::vector<std::pair<int, double>>& d, bool use_total) const;
  std::vector<std::pair<int, double>> to_vec(const ResMap& m);
  double utilization(const NodeRes& n) const;
  std::vector<std::string> place_bundles(const std::vector<ResMap>& bundles, int strategy,
                                         bool use_total);

  std::unordered_map<std::string, int> res_ids_;
  std::vector<std::string> res_names_;
  std::vector<NodeRes> nodes_;
  std::unordered_map<std::string, int> node_idx_;
  struct PgRecord {
    std::vector<std::string> nodes;
    std::vector<ResMap> bundles;
  };
  std::unordered_map<std::string, PgRecord> pgs_;
  double spread_threshold_;
  size_t rr_ = 0;
};

}  // namespace caamd_rt
