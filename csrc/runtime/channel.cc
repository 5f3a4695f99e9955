#include "channel.h"

#include <errno.h>
#include <fcntl.h>
#include <linux/futex.h>
#include <sched.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <sys/syscall.h>
#include <time.h>
#include <unistd.h>

#include <chrono>
#include <stdexcept>

namespace caamd_rt {

static constexpr uint64_t kMagic = 0x43414d4443484e31ull;  // "CAMDCHN1"
static constexpr uint64_t kHeaderBytes = 4096;
static_assert(sizeof(ChannelHeader) <= kHeaderBytes, "channel header too large");

static uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

static std::string shm_path(const std::string& name) {
  return "/dev/shm/" + (name[0] == '/' ? name.substr(1) : name);
}

Channel::Channel(const std::string& name, bool create, uint32_t num_readers, uint32_t num_slots,
                 uint64_t slot_bytes)
    : name_(name) {
  const std::string path = shm_path(name);
  if (create) {
    if (num_readers < 1 || num_readers > (uint32_t)kMaxReaders) throw std::invalid_argument("num_readers");
    if (num_slots < 1) throw std::invalid_argument("num_slots");
    stride_ = round_up(sizeof(SlotHdr) + slot_bytes, 64);
    map_bytes_ = kHeaderBytes + stride_ * num_slots;
    fd_ = ::open(path.c_str(), O_RDWR | O_CREAT | O_TRUNC, 0600);
    if (fd_ < 0) throw std::runtime_error("channel open " + path + ": " + strerror(errno));
    if (::ftruncate(fd_, (off_t)map_bytes_) != 0) {
      ::close(fd_);
      throw std::runtime_error("channel ftruncate: " + std::string(strerror(errno)));
    }
  } else {
    fd_ = ::open(path.c_str(), O_RDWR);
    if (fd_ < 0) throw std::runtime_error("channel attach " + path + ": " + strerror(errno));
    struct stat st;
    if (::fstat(fd_, &st) != 0 || (uint64_t)st.st_size < kHeaderBytes) {
      ::close(fd_);
      throw std::runtime_error("channel attach: bad file " + path);
    }
    map_bytes_ = (uint64_t)st.st_size;
  }
  void* p = ::mmap(nullptr, map_bytes_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
  if (p == MAP_FAILED) {
    ::close(fd_);
    throw std::runtime_error("channel mmap: " + std::string(strerror(errno)));
  }
  base_ = (uint8_t*)p;
  hdr_ = (ChannelHeader*)base_;
  if (create) {
    memset(base_, 0, kHeaderBytes);
    new (hdr_) ChannelHeader();
    hdr_->num_readers = num_readers;
    hdr_->num_slots = num_slots;
    hdr_->slot_bytes = slot_bytes;
    hdr_->total_bytes = map_bytes_;
    std::atomic_thread_fence(std::memory_order_release);
    hdr_->magic = kMagic;
  } else {
    if (hdr_->magic != kMagic) {
      ::munmap(base_, map_bytes_);
      ::close(fd_);
      throw std::runtime_error("channel attach: not a channel " + path);
    }
    stride_ = round_up(sizeof(SlotHdr) + hdr_->slot_bytes, 64);
  }
}

Channel::~Channel() {
  if (base_) ::munmap(base_, map_bytes_);
  if (fd_ >= 0) ::close(fd_);
}

uint8_t* Channel::slot(uint64_t seq) const {
  return base_ + kHeaderBytes + (seq % hdr_->num_slots) * stride_;
}

uint64_t Channel::min_read() const {
  uint64_t m = UINT64_MAX;
  for (uint32_t r = 0; r < hdr_->num_readers; ++r) {
    const uint64_t v = hdr_->read_seq[r].load(std::memory_order_acquire);
    m = v < m ? v : m;
  }
  return m;
}

void Channel::notify() {
  hdr_->futex.fetch_add(1, std::memory_order_acq_rel);
  if (hdr_->waiters.load(std::memory_order_acquire) != 0)
    syscall(SYS_futex, (uint32_t*)&hdr_->futex, FUTEX_WAKE, INT32_MAX, nullptr, nullptr, 0);
}

template <class Pred>
bool Channel::wait_until(Pred pred, double timeout_s) {
  using clk = std::chrono::steady_clock;
  const auto t0 = clk::now();
  // phase 1: spin ~20 us (a pipelined partner usually publishes within that)
  for (int i = 0; i < 2000; ++i) {
    if (pred()) return true;
    if ((i & 63) == 63) sched_yield();
  }
  // phase 2: futex sleep, re-checking the predicate after registering as a waiter
  while (true) {
    const uint32_t f = hdr_->futex.load(std::memory_order_acquire);
    if (pred()) return true;
    double left = 0.05;
    if (timeout_s >= 0) {
      const double el = std::chrono::duration<double>(clk::now() - t0).count();
      if (el >= timeout_s) return pred();
      left = std::min(left, timeout_s - el);
    }
    struct timespec ts;
    ts.tv_sec = (time_t)left;
    ts.tv_nsec = (long)((left - (double)ts.tv_sec) * 1e9);
    hdr_->waiters.fetch_add(1, std::memory_order_acq_rel);
    if (!pred()) syscall(SYS_futex, (uint32_t*)&hdr_->futex, FUTEX_WAIT, f, &ts, nullptr, 0);
    hdr_->waiters.fetch_sub(1, std::memory_order_acq_rel);
  }
}

int Channel::write(const void* data, uint64_t len, uint64_t flags, double timeout_s) {
  if (len > hdr_->slot_bytes) return -3;
  if (closed()) return -2;
  const uint64_t seq = hdr_->write_seq.load(std::memory_order_relaxed);
  const uint32_t ns = hdr_->num_slots;
  bool ok = wait_until([&] { return closed() || seq - min_read() < ns; }, timeout_s);
  if (!ok) return -1;
  if (closed()) return -2;
  uint8_t* s = slot(seq);
  SlotHdr* sh = (SlotHdr*)s;
  sh->len = len;
  sh->flags = flags;
  if (len) memcpy(s + sizeof(SlotHdr), data, len);
  hdr_->write_seq.store(seq + 1, std::memory_order_release);
  notify();
  return 0;
}

int Channel::begin_read(uint32_t reader, const uint8_t** data, uint64_t* len, uint64_t* flags,
                        double timeout_s) {
  if (reader >= hdr_->num_readers) return -4;
  const uint64_t mine = hdr_->read_seq[reader].load(std::memory_order_relaxed);
  auto avail = [&] { return hdr_->write_seq.load(std::memory_order_acquire) > mine; };
  bool ok = wait_until([&] { return avail() || closed(); }, timeout_s);
  if (!ok) return -1;
  if (!avail()) return -2;  // closed and nothing left for this reader
  const uint8_t* s = slot(mine);
  const SlotHdr* sh = (const SlotHdr*)s;
  *len = sh->len;
  *flags = sh->flags;
  *data = s + sizeof(SlotHdr);
  return 0;
}

void Channel::end_read(uint32_t reader) {
  hdr_->read_seq[reader].fetch_add(1, std::memory_order_acq_rel);
  notify();
}

void Channel::close() {
  hdr_->closed.store(1, std::memory_order_release);
  notify();
}

void Channel::unlink() { ::unlink(shm_path(name_).c_str()); }

}  // namespace caamd_rt
