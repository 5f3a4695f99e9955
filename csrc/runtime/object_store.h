// Shared-memory immutable object store (the Plasma role, reference:
// src/ray/object_manager/plasma/). One arena file in /dev/shm per node, mapped by
// every process of the node; all metadata (allocator + object table) lives IN the
// arena so a worker resolves a sealed object with no round trip to the raylet.
//
// Layout: [Header | object table (open addressing) | data region]
//  * data region: boundary-tag allocator, 64-byte aligned payloads (so numpy /
//    torch views of object buffers are aligned for vector loads and for
//    hipHostRegister when an object is staged to HBM), explicit free list with
//    coalescing; LRU-ish eviction is driven by the owner (Python side).
//  * concurrency: one robust process-shared mutex (a crashed worker holding it
//    is recovered with EOWNERDEAD), operations are O(1) expected.
#pragma once
#include <pthread.h>
#include <stdint.h>

#include <atomic>
#include <string>
#include <thread>
#include <vector>

namespace caamd_rt {

constexpr int kIdBytes = 24;
constexpr uint64_t kAlign = 64;

struct ObjectEntry {
  uint8_t id[kIdBytes];
  uint64_t offset;     // payload offset from arena base
  uint64_t size;       // payload bytes
  uint64_t meta;       // user metadata word (e.g. format flags)
  uint32_t state;      // 0 empty, 1 created, 2 sealed, 3 tombstone, 4 deleted-but-pinned
  int32_t pins;        // readers holding views (advisory, for eviction)
  uint64_t lru;        // last access tick
};

struct BlockHdr {  // 64 bytes, precedes every block (free or used)
  uint64_t size;       // whole block incl. header
  uint64_t prev_size;  // size of physically previous block (0 = first)
  uint64_t next_free;  // free-list links (offsets of block headers), valid when free
  uint64_t prev_free;
  uint32_t free;
  uint32_t pad0;
  uint64_t pad[3];
};
static_assert(sizeof(BlockHdr) == 64, "BlockHdr must be 64 bytes");

struct Header {
  uint64_t magic;
  uint64_t total_size;
  uint64_t table_offset;
  uint64_t table_capacity;  // power of two
  uint64_t data_offset;
  uint64_t data_size;
  uint64_t free_head;  // offset of first free block header, 0 = none
  uint64_t used_bytes;
  uint64_t num_objects;
  uint64_t tick;
  pthread_mutex_t mu;
  // copy threads currently running in copy_in() across every process of the node:
  // concurrent large puts share one node-wide budget instead of each spawning its
  // own full set (10 putters x 4 threads on 8 cores thrashed the memory system).
  // One slot per in-flight claim, packed (pid << 32 | threads) so that a claim is
  // taken, released and reclaimed by a single 64-bit CAS: a claim whose process died
  // mid-put (SIGKILL, OOM kill) is reclaimed by the next claimer instead of leaking
  // its threads out of the budget for the life of the store.
  static constexpr int kCopyClaims = 64;
  uint64_t copy_claims[kCopyClaims];
  uint32_t copy_threads_budget;
  uint32_t pad_claims;
};

class ObjectStore {
 public:
  // create=true: make a new arena (unlinks an existing file of that name)
  ObjectStore(const std::string& name, uint64_t capacity, uint64_t table_capacity, bool create);
  ~ObjectStore();

  // returns payload offset, or -1 if no space, -2 if id exists
  int64_t create(const std::string& id, uint64_t size, uint64_t meta);
  bool seal(const std::string& id);
  // returns (offset, size, meta) if sealed; offset -1 otherwise
  bool lookup(const std::string& id, uint64_t* off, uint64_t* size, uint64_t* meta, bool pin);
  void unpin(const std::string& id);
  bool contains(const std::string& id);
  bool remove(const std::string& id);  // frees the payload
  bool abort(const std::string& id);   // remove an unsealed object

  uint64_t capacity() const { return hdr_->data_size; }
  uint64_t map_size() const { return map_size_; }
  uint64_t used() const { return hdr_->used_bytes; }
  uint64_t num_objects() const { return hdr_->num_objects; }
  uint8_t* base() const { return base_; }
  const std::string& name() const { return name_; }
  // ids of sealed, unpinned objects in least-recently-used order (eviction candidates)
  std::vector<std::string> lru_candidates(uint64_t max_count);
  std::vector<std::string> list_ids();
  uint64_t largest_free();
  void unlink();
  // Copy n bytes into the arena at `off` with up to `threads` threads (large
  // puts: first-touch page faults of fresh shm pages cost ~1 GB/s on one core;
  // spread over cores they scale, and faulted pages copy at memcpy speed).
  void copy_in(uint64_t off, const void* src, uint64_t n, int threads);
  // copy threads claimed node-wide right now (sum over the live claim slots)
  uint32_t copy_threads_claimed();
  // test hook: plant a claim as process `pid` would (a dead pid models a SIGKILLed putter)
  void debug_plant_claim(uint32_t pid, uint32_t threads) {
    for (int i = 0; i < Header::kCopyClaims; ++i) {
      uint64_t e = 0;
      if (__atomic_compare_exchange_n(&hdr_->copy_claims[i], &e, ((uint64_t)pid << 32) | threads, false,
                                      __ATOMIC_ACQ_REL, __ATOMIC_RELAXED))
        return;
    }
  }
  // Touch (fault in) the first `max_bytes` of the data region in a detached
  // background thread, so the first large puts do not pay page faults.
  void prefault_async(uint64_t max_bytes);

 private:
  uint32_t claim_copy_threads(uint32_t want, uint32_t budget);
  void lock();
  void unlock();
  ObjectEntry* find(const uint8_t* id, bool for_insert);
  uint64_t alloc(uint64_t size);
  void free_block(uint64_t blk);
  void fl_insert(uint64_t blk);
  void fl_remove(uint64_t blk);
  BlockHdr* B(uint64_t off) const { return reinterpret_cast<BlockHdr*>(base_ + off); }

  std::string name_;
  int fd_ = -1;
  uint8_t* base_ = nullptr;
  uint64_t map_size_ = 0;
  Header* hdr_ = nullptr;
  ObjectEntry* table_ = nullptr;
  std::thread prefault_;
  std::atomic<bool> stop_prefault_{false};
};

}  // namespace caamd_rt
