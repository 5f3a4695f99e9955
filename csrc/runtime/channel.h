// Shared-memory message channel for compiled graphs (the role of the reference's
// python/ray/experimental/channel/shared_memory_channel.py + the mutable-object
// manager in src/ray/core_worker/experimental_mutable_object_manager.cc).
//
// One writer, N readers, a ring of `num_slots` fixed-size slots in one /dev/shm
// file. Every reader sees every message (broadcast): slot `seq % num_slots` may be
// overwritten only after ALL readers have consumed `seq`. Sequence counters are
// 64-bit atomics in the mapped header, so writer and readers in different
// processes synchronize with acquire/release ordering and no lock. Blocking waits
// spin briefly (the hot path of a pipelined graph: the partner publishes within
// microseconds) and then sleep on a shared futex word that every publish/consume
// bumps, so an idle pipeline costs no CPU.
//
// Layout: [Header (4 KiB) | slot 0 | slot 1 | ...], slot = [SlotHdr (64 B) | data].
#pragma once
#include <stdint.h>

#include <atomic>
#include <string>

namespace caamd_rt {

constexpr int kMaxReaders = 64;

struct alignas(64) ChannelHeader {
  uint64_t magic;
  uint32_t num_readers;
  uint32_t num_slots;
  uint64_t slot_bytes;  // payload capacity of one slot
  uint64_t total_bytes;
  alignas(64) std::atomic<uint64_t> write_seq;  // messages published
  alignas(64) std::atomic<uint32_t> futex;      // bumped on every state change
  std::atomic<uint32_t> waiters;
  std::atomic<uint32_t> closed;
  alignas(64) std::atomic<uint64_t> read_seq[kMaxReaders];  // messages consumed, per reader
};

struct alignas(64) SlotHdr {
  uint64_t len;
  uint64_t flags;  // user tag (e.g. "payload is an object-store reference")
};

class Channel {
 public:
  // create=true: make (or truncate) the shm file; otherwise attach to it.
  Channel(const std::string& name, bool create, uint32_t num_readers, uint32_t num_slots,
          uint64_t slot_bytes);
  ~Channel();
  Channel(const Channel&) = delete;
  Channel& operator=(const Channel&) = delete;

  // Publish one message. Blocks while the ring is full. Returns 0 ok, -1 timeout,
  // -2 closed, -3 too large.
  int write(const void* data, uint64_t len, uint64_t flags, double timeout_s);
  // Wait for the next message of `reader`; on success *data points INTO the slot
  // (valid until end_read). Returns 0 ok, -1 timeout, -2 closed and drained.
  int begin_read(uint32_t reader, const uint8_t** data, uint64_t* len, uint64_t* flags,
                 double timeout_s);
  void end_read(uint32_t reader);
  void close();
  void unlink();

  bool closed() const { return hdr_->closed.load(std::memory_order_acquire) != 0; }
  uint32_t num_readers() const { return hdr_->num_readers; }
  uint32_t num_slots() const { return hdr_->num_slots; }
  uint64_t slot_bytes() const { return hdr_->slot_bytes; }
  uint64_t write_seq() const { return hdr_->write_seq.load(std::memory_order_acquire); }
  uint64_t read_seq(uint32_t r) const { return hdr_->read_seq[r].load(std::memory_order_acquire); }
  const std::string& name() const { return name_; }

 private:
  uint8_t* slot(uint64_t seq) const;
  uint64_t min_read() const;
  // wait until pred() is true; false on timeout
  template <class Pred>
  bool wait_until(Pred pred, double timeout_s);
  void notify();

  std::string name_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  uint64_t map_bytes_ = 0;
  ChannelHeader* hdr_ = nullptr;
  uint64_t stride_ = 0;
};

}  // namespace caamd_rt
