// Durable table store for the head's GCS state (reference role:
// src/ray/gcs/store_client/redis_store_client.h:107 -- the GCS persists its
// tables to an external Redis so a restarted GCS can reload them).
//
// Here the backing store is a local append-only log file (single node / shared
// filesystem): every put / delete appends one checksummed record; opening the
// store replays the log into in-memory hash tables and truncates a torn tail
// (a record cut short or failing its CRC by a crash mid-write). When dead
// records outweigh live ones the log is compacted into a fresh file that is
// renamed over the old one, so the on-disk size stays O(live data).
#pragma once

#include <cstdint>
#include <mutex>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

namespace caamd_rt {

class GcsStore {
 public:
  // Opens (creating if needed) the log at `path` and replays it.
  explicit GcsStore(const std::string& path, bool fsync_each = false);
  ~GcsStore();
  GcsStore(const GcsStore&) = delete;
  GcsStore& operator=(const GcsStore&) = delete;

  void put(const std::string& table, const std::string& key, const std::string& value);
  bool del(const std::string& table, const std::string& key);
  bool get(const std::string& table, const std::string& key, std::string* value) const;
  std::vector<std::string> keys(const std::string& table) const;
  std::vector<std::pair<std::string, std::string>> items(const std::string& table) const;
  std::vector<std::string> tables() const;
  void clear_table(const std::string& table);

  void sync();     // fsync the log
  void compact();  // rewrite the log with live records only
  uint64_t log_bytes() const { return log_bytes_; }
  uint64_t live_bytes() const { return live_bytes_; }
  uint64_t records_replayed() const { return replayed_; }
  uint64_t torn_bytes_dropped() const { return torn_; }
  const std::string& path() const { return path_; }
  // Test hook: the next append writes only `bytes` bytes of its record and then
  // fails as a short write / ENOSPC would (-1 disables).
  void inject_write_fault(int64_t bytes) { fault_after_ = bytes; }

 private:
  void replay();
  void append(uint8_t op, const std::string& table, const std::string& key, const std::string& value);
  void maybe_compact();
  static std::string encode(uint8_t op, const std::string& table, const std::string& key,
                            const std::string& value);

  std::string path_;
  bool fsync_each_;
  int fd_ = -1;
  uint64_t log_bytes_ = 0, live_bytes_ = 0, replayed_ = 0, torn_ = 0;
  int64_t fault_after_ = -1;
  std::unordered_map<std::string, std::unordered_map<std::string, std::string>> tables_;
  mutable std::mutex mu_;
};

}  // namespace caamd_rt
