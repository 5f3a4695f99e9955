// Append-only, checksummed log store for GCS tables (see gcs_store.h).
//
// Record layout (little endian):
//   u32 magic 'GCS1' | u8 op (1 put, 2 del, 3 clear-table) | u32 table_len |
//   u32 key_len | u32 value_len | table | key | value | u32 crc32(op .. value)
#include <algorithm>
#include "gcs_store.h"

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <cerrno>
#include <cstring>
#include <stdexcept>

namespace caamd_rt {

namespace {

constexpr uint32_t kMagic = 0x31534347u;  // "GCS1"
constexpr size_t kHeader = 4 + 1 + 4 + 4 + 4;

uint32_t crc32(const uint8_t* p, size_t n, uint32_t crc = 0) {
  static uint32_t table[256];
  static bool init = [] {
    for (uint32_t i = 0; i < 256; ++i) {
      uint32_t c = i;
      for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
      table[i] = c;
    }
    return true;
  }();
  (void)init;
  crc = ~crc;
  for (size_t i = 0; i < n; ++i) crc = table[(crc ^ p[i]) & 0xff] ^ (crc >> 8);
  return ~crc;
}

void put_u32(std::string& s, uint32_t v) {
  char b[4];
  std::memcpy(b, &v, 4);
  s.append(b, 4);
}
uint32_t get_u32(const uint8_t* p) {
  uint32_t v;
  std::memcpy(&v, p, 4);
  return v;
}

void write_all(int fd, const std::string& s) {
  size_t off = 0;
  while (off < s.size()) {
    ssize_t n = ::write(fd, s.data() + off, s.size() - off);
    if (n < 0) {
      if (errno == EINTR) continue;
      throw std::runtime_error(std::string("GcsStore: write failed: ") + std::strerror(errno));
    }
    off += (size_t)n;
  }
}

size_t record_size(const std::string& t, const std::string& k, const std::string& v) {
  return kHeader + t.size() + k.size() + v.size() + 4;
}

}  // namespace

std::string GcsStore::encode(uint8_t op, const std::string& table, const std::string& key,
                             const std::string& value) {
  std::string r;
  r.reserve(record_size(table, key, value));
  put_u32(r, kMagic);
  r.push_back((char)op);
  put_u32(r, (uint32_t)table.size());
  put_u32(r, (uint32_t)key.size());
  put_u32(r, (uint32_t)value.size());
  r += table;
  r += key;
  r += value;
  put_u32(r, crc32((const uint8_t*)r.data() + 4, r.size() - 4));
  return r;
}

GcsStore::GcsStore(const std::string& path, bool fsync_each) : path_(path), fsync_each_(fsync_each) {
  fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_CLOEXEC, 0600);
  if (fd_ < 0) throw std::runtime_error("GcsStore: cannot open " + path + ": " + std::strerror(errno));
  replay();
}

GcsStore::~GcsStore() {
  if (fd_ >= 0) ::close(fd_);
}

void GcsStore::replay() {
  struct stat st;
  if (::fstat(fd_, &st) != 0) throw std::runtime_error("GcsStore: fstat failed");
  std::string buf((size_t)st.st_size, '\0');
  size_t got = 0;
  while (got < buf.size()) {
    ssize_t n = ::pread(fd_, &buf[got], buf.size() - got, (off_t)got);
    if (n <= 0) {
      if (n < 0 && errno == EINTR) continue;
      break;
    }
    got += (size_t)n;
  }
  buf.resize(got);
  const uint8_t* p = (const uint8_t*)buf.data();
  size_t off = 0, good = 0;
  while (off + kHeader + 4 <= buf.size()) {
    if (get_u32(p + off) != kMagic) break;
    const uint8_t op = p[off + 4];
    const uint32_t tl = get_u32(p + off + 5), kl = get_u32(p + off + 9), vl = get_u32(p + off + 13);
    const size_t total = kHeader + (size_t)tl + kl + vl + 4;
    if (off + total > buf.size()) break;  // torn tail
    const uint32_t want = get_u32(p + off + total - 4);
    if (crc32(p + off + 4, total - 8) != want) break;
    std::string t((const char*)p + off + kHeader, tl);
    std::string k((const char*)p + off + kHeader + tl, kl);
    std::string v((const char*)p + off + kHeader + tl + kl, vl);
    auto& tab = tables_[t];
    if (op == 1) {
      auto it = tab.find(k);
      if (it != tab.end()) live_bytes_ -= record_size(t, k, it->second);
      live_bytes_ += total;
      tab[k] = std::move(v);
    } else if (op == 2) {
      auto it = tab.find(k);
      if (it != tab.end()) {
        live_bytes_ -= record_size(t, k, it->second);
        tab.erase(it);
      }
    } else if (op == 3) {
      for (auto& kv : tab) live_bytes_ -= record_size(t, kv.first, kv.second);
      tab.clear();
    } else {
      break;
    }
    off += total;
    good = off;
    ++replayed_;
  }
  torn_ = buf.size() - good;
  if (torn_ > 0 && ::ftruncate(fd_, (off_t)good) != 0)
    throw std::runtime_error("GcsStore: cannot truncate torn tail");
  log_bytes_ = good;
  ::lseek(fd_, (off_t)good, SEEK_SET);
}

void GcsStore::append(uint8_t op, const std::string& table, const std::string& key, const std::string& value) {
  const std::string r = encode(op, table, key, value);
  try {
    if (fault_after_ >= 0) {  // test hook: a short write, then the failure
      const size_t n = std::min((size_t)fault_after_, r.size());
      fault_after_ = -1;
      write_all(fd_, r.substr(0, n));
      throw std::runtime_error("GcsStore: write failed: injected short write");
    }
    write_all(fd_, r);
  } catch (...) {
    // A partial record must not stay in the middle of the log: replay stops at the
    // first bad record, so every later append behind it would be lost on restart.
    // Cut the file back to the last whole record and put the offset there.
    if (::ftruncate(fd_, (off_t)log_bytes_) != 0) {
      throw std::runtime_error("GcsStore: write failed and the partial record could not be removed");
    }
    ::lseek(fd_, (off_t)log_bytes_, SEEK_SET);
    throw;
  }
  if (fsync_each_) ::fdatasync(fd_);
  log_bytes_ += r.size();
}

void GcsStore::put(const std::string& table, const std::string& key, const std::string& value) {
  std::lock_guard<std::mutex> g(mu_);
  append(1, table, key, value);
  auto& tab = tables_[table];
  auto it = tab.find(key);
  if (it != tab.end()) live_bytes_ -= record_size(table, key, it->second);
  live_bytes_ += record_size(table, key, value);
  tab[key] = value;
  maybe_compact();
}

bool GcsStore::del(const std::string& table, const std::string& key) {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  if (t == tables_.end()) return false;
  auto it = t->second.find(key);
  if (it == t->second.end()) return false;
  append(2, table, key, std::string());
  live_bytes_ -= record_size(table, key, it->second);
  t->second.erase(it);
  maybe_compact();
  return true;
}

void GcsStore::clear_table(const std::string& table) {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  if (t == tables_.end() || t->second.empty()) return;
  append(3, table, std::string(), std::string());
  for (auto& kv : t->second) live_bytes_ -= record_size(table, kv.first, kv.second);
  t->second.clear();
  maybe_compact();
}

bool GcsStore::get(const std::string& table, const std::string& key, std::string* value) const {
  std::lock_guard<std::mutex> g(mu_);
  auto t = tables_.find(table);
  if (t == tables_.end()) return false;
  auto it = t->second.find(key);
  if (it == t->second.end()) return false;
  *value = it->second;
  return true;
}

std::vector<std::string> GcsStore::keys(const std::string& table) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  auto t = tables_.find(table);
  if (t != tables_.end())
    for (auto& kv : t->second) out.push_back(kv.first);
  return out;
}

std::vector<std::pair<std::string, std::string>> GcsStore::items(const std::string& table) const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::pair<std::string, std::string>> out;
  auto t = tables_.find(table);
  if (t != tables_.end())
    for (auto& kv : t->second) out.emplace_back(kv.first, kv.second);
  return out;
}

std::vector<std::string> GcsStore::tables() const {
  std::lock_guard<std::mutex> g(mu_);
  std::vector<std::string> out;
  for (auto& t : tables_)
    if (!t.second.empty()) out.push_back(t.first);
  return out;
}

void GcsStore::sync() {
  std::lock_guard<std::mutex> g(mu_);
  ::fsync(fd_);
}

void GcsStore::maybe_compact() {
  // dead records outweigh live ones (and the log is worth rewriting)
  if (log_bytes_ > (1u << 20) && log_bytes_ > 2 * live_bytes_) {
    mu_.unlock();
    try {
      compact();
    } catch (...) {
      mu_.lock();
      throw;
    }
    mu_.lock();
  }
}

void GcsStore::compact() {
  std::lock_guard<std::mutex> g(mu_);
  const std::string tmp = path_ + ".compact";
  int nfd = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0600);
  if (nfd < 0) throw std::runtime_error("GcsStore: cannot create " + tmp);
  uint64_t bytes = 0;
  try {
    std::string chunk;
    for (auto& t : tables_)
      for (auto& kv : t.second) {
        chunk += encode(1, t.first, kv.first, kv.second);
        if (chunk.size() > (1u << 20)) {
          write_all(nfd, chunk);
          bytes += chunk.size();
          chunk.clear();
        }
      }
    write_all(nfd, chunk);
    bytes += chunk.size();
    ::fsync(nfd);
  } catch (...) {
    ::close(nfd);
    ::unlink(tmp.c_str());
    throw;
  }
  if (::rename(tmp.c_str(), path_.c_str()) != 0) {
    ::close(nfd);
    throw std::runtime_error("GcsStore: rename failed");
  }
  ::close(fd_);
  fd_ = nfd;
  ::lseek(fd_, 0, SEEK_END);
  log_bytes_ = bytes;
  live_bytes_ = bytes;
}

}  // namespace caamd_rt
