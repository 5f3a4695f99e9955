#include "object_store.h"

#include <immintrin.h>

#include <errno.h>
#include <signal.h>
#include <fcntl.h>
#include <string.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <stdexcept>
#include <thread>
#include <vector>

namespace caamd_rt {

static constexpr uint64_t kMagic = 0x43414d444f424a31ull;  // "CAMDOBJ1"
static constexpr uint64_t kMinBlock = 128;

static inline uint64_t round_up(uint64_t x, uint64_t a) { return (x + a - 1) / a * a; }

static inline uint64_t hash_id(const uint8_t* id) {
  uint64_t h = 1469598103934665603ull;
  for (int i = 0; i < kIdBytes; ++i) {
    h ^= id[i];
    h *= 1099511628211ull;
  }
  return h;
}

ObjectStore::ObjectStore(const std::string& name, uint64_t capacity, uint64_t table_capacity,
                         bool create)
    : name_(name) {
  if (create) {
    uint64_t tc = 1;
    while (tc < table_capacity) tc <<= 1;
    const uint64_t table_off = round_up(sizeof(Header), 4096);
    const uint64_t data_off = round_up(table_off + tc * sizeof(ObjectEntry), 4096);
    const uint64_t data_size = round_up(std::max<uint64_t>(capacity, 1 << 20), kAlign);
    map_size_ = data_off + data_size;
    shm_unlink(name.c_str());
    fd_ = shm_open(name.c_str(), O_CREAT | O_RDWR | O_EXCL, 0600);
    if (fd_ < 0) throw std::runtime_error("shm_open(create) failed: " + std::string(strerror(errno)));
    if (ftruncate(fd_, (off_t)map_size_) != 0) {
      close(fd_);
      shm_unlink(name.c_str());
      throw std::runtime_error("ftruncate failed: " + std::string(strerror(errno)));
    }
    base_ = (uint8_t*)mmap(nullptr, map_size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    hdr_ = reinterpret_cast<Header*>(base_);
    hdr_->total_size = map_size_;
    hdr_->table_offset = table_off;
    hdr_->table_capacity = tc;
    hdr_->data_offset = data_off;
    hdr_->data_size = data_size;
    hdr_->used_bytes = 0;
    hdr_->num_objects = 0;
    hdr_->tick = 0;
    for (int i = 0; i < Header::kCopyClaims; ++i) hdr_->copy_claims[i] = 0;
    hdr_->copy_threads_budget = std::max(2u, std::thread::hardware_concurrency() / 2);
    pthread_mutexattr_t a;
    pthread_mutexattr_init(&a);
    pthread_mutexattr_setpshared(&a, PTHREAD_PROCESS_SHARED);
    pthread_mutexattr_setrobust(&a, PTHREAD_MUTEX_ROBUST);
    pthread_mutex_init(&hdr_->mu, &a);
    pthread_mutexattr_destroy(&a);
    table_ = reinterpret_cast<ObjectEntry*>(base_ + table_off);
    // one free block spanning the data region
    BlockHdr* b = B(data_off);
    b->size = data_size;
    b->prev_size = 0;
    b->free = 1;
    b->next_free = b->prev_free = 0;
    hdr_->free_head = data_off;
    __atomic_store_n(&hdr_->magic, kMagic, __ATOMIC_RELEASE);
  } else {
    fd_ = shm_open(name.c_str(), O_RDWR, 0600);
    if (fd_ < 0) throw std::runtime_error("shm_open(attach) failed: " + std::string(strerror(errno)));
    struct stat st;
    fstat(fd_, &st);
    map_size_ = (uint64_t)st.st_size;
    base_ = (uint8_t*)mmap(nullptr, map_size_, PROT_READ | PROT_WRITE, MAP_SHARED, fd_, 0);
    if (base_ == MAP_FAILED) throw std::runtime_error("mmap failed");
    hdr_ = reinterpret_cast<Header*>(base_);
    if (__atomic_load_n(&hdr_->magic, __ATOMIC_ACQUIRE) != kMagic)
      throw std::runtime_error("object store arena has a bad magic");
    table_ = reinterpret_cast<ObjectEntry*>(base_ + hdr_->table_offset);
  }
}

ObjectStore::~ObjectStore() {
  stop_prefault_.store(true);
  if (prefault_.joinable()) prefault_.join();  // never unmap under the prefault thread
  if (base_ && base_ != MAP_FAILED) munmap(base_, map_size_);
  if (fd_ >= 0) close(fd_);
}

void ObjectStore::unlink() { shm_unlink(name_.c_str()); }

void ObjectStore::lock() {
  int r = pthread_mutex_lock(&hdr_->mu);
  if (r == EOWNERDEAD) pthread_mutex_consistent(&hdr_->mu);  // a worker died holding it
}
void ObjectStore::unlock() { pthread_mutex_unlock(&hdr_->mu); }

ObjectEntry* ObjectStore::find(const uint8_t* id, bool for_insert) {
  const uint64_t mask = hdr_->table_capacity - 1;
  uint64_t i = hash_id(id) & mask;
  ObjectEntry* tomb = nullptr;
  for (uint64_t n = 0; n <= mask; ++n, i = (i + 1) & mask) {
    ObjectEntry* e = &table_[i];
    if (e->state == 0) return for_insert ? (tomb ? tomb : e) : nullptr;
    if (e->state == 3) {
      if (!tomb) tomb = e;
      continue;
    }
    if (memcmp(e->id, id, kIdBytes) == 0) return e;
  }
  return for_insert ? tomb : nullptr;
}

void ObjectStore::fl_insert(uint64_t blk) {
  BlockHdr* b = B(blk);
  b->free = 1;
  b->prev_free = 0;
  b->next_free = hdr_->free_head;
  if (hdr_->free_head) B(hdr_->free_head)->prev_free = blk;
  hdr_->free_head = blk;
}

void ObjectStore::fl_remove(uint64_t blk) {
  BlockHdr* b = B(blk);
  if (b->prev_free) B(b->prev_free)->next_free = b->next_free;
  else hdr_->free_head = b->next_free;
  if (b->next_free) B(b->next_free)->prev_free = b->prev_free;
  b->free = 0;
  b->next_free = b->prev_free = 0;
}

uint64_t ObjectStore::alloc(uint64_t size) {
  const uint64_t need = std::max(kMinBlock, round_up(size + sizeof(BlockHdr), kAlign));
  const uint64_t end = hdr_->data_offset + hdr_->data_size;
  // best fit among the first few candidates (bounded scan keeps it O(1)-ish)
  uint64_t best = 0, best_size = ~0ull;
  int scanned = 0;
  for (uint64_t f = hdr_->free_head; f; f = B(f)->next_free) {
    const uint64_t s = B(f)->size;
    if (s >= need && s < best_size) {
      best = f;
      best_size = s;
      if (s - need < kMinBlock) break;
    }
    if (best && ++scanned > 64) break;
  }
  if (!best) return 0;
  fl_remove(best);
  BlockHdr* b = B(best);
  if (b->size - need >= kMinBlock) {
    const uint64_t rest = best + need;
    BlockHdr* r = B(rest);
    r->size = b->size - need;
    r->prev_size = need;
    const uint64_t nxt = rest + r->size;
    if (nxt < end) B(nxt)->prev_size = r->size;
    b->size = need;
    fl_insert(rest);
  }
  b->free = 0;
  hdr_->used_bytes += b->size;
  return best;
}

void ObjectStore::free_block(uint64_t blk) {
  const uint64_t end = hdr_->data_offset + hdr_->data_size;
  BlockHdr* b = B(blk);
  hdr_->used_bytes -= b->size;
  // coalesce with next
  uint64_t nxt = blk + b->size;
  if (nxt < end && B(nxt)->free) {
    fl_remove(nxt);
    b->size += B(nxt)->size;
  }
  // coalesce with prev
  if (b->prev_size) {
    const uint64_t prv = blk - b->prev_size;
    if (B(prv)->free) {
      fl_remove(prv);
      B(prv)->size += b->size;
      blk = prv;
      b = B(prv);
    }
  }
  nxt = blk + b->size;
  if (nxt < end) B(nxt)->prev_size = b->size;
  fl_insert(blk);
}

int64_t ObjectStore::create(const std::string& id, uint64_t size, uint64_t meta) {
  if (id.size() != kIdBytes) throw std::invalid_argument("object id must be 24 bytes");
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), true);
  if (!e) {
    unlock();
    return -3;  // table full
  }
  if (e->state == 1 || e->state == 2 || e->state == 4 || e->state == 5) {
    if (memcmp(e->id, id.data(), kIdBytes) == 0) {
      unlock();
      return -2;
    }
  }
  const uint64_t blk = alloc(size);
  if (!blk) {
    unlock();
    return -1;
  }
  memcpy(e->id, id.data(), kIdBytes);
  e->offset = blk + sizeof(BlockHdr);
  e->size = size;
  e->meta = meta;
  e->state = 1;
  e->pins = 0;
  e->lru = ++hdr_->tick;
  hdr_->num_objects++;
  const int64_t off = (int64_t)e->offset;
  unlock();
  return off;
}

bool ObjectStore::seal(const std::string& id) {
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), false);
  bool ok = e && e->state == 1;
  if (ok) {
    __atomic_store_n(&e->state, 2u, __ATOMIC_RELEASE);
  } else if (e && e->state == 5) {
    // removed while its creator was still writing: the block was kept for the
    // writer; free it now that the copy-in is over
    free_block(e->offset - sizeof(BlockHdr));
    e->state = 3;
  }
  unlock();
  return ok;
}

bool ObjectStore::lookup(const std::string& id, uint64_t* off, uint64_t* size, uint64_t* meta,
                         bool pin) {
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), false);
  bool ok = e && e->state == 2;
  if (ok) {
    *off = e->offset;
    *size = e->size;
    *meta = e->meta;
    e->lru = ++hdr_->tick;
    if (pin) e->pins++;
  }
  unlock();
  return ok;
}

void ObjectStore::unpin(const std::string& id) {
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), false);
  if (e && e->pins > 0) {
    e->pins--;
    if (e->pins == 0 && e->state == 4) {  // deletion was deferred while readers held views
      free_block(e->offset - sizeof(BlockHdr));
      e->state = 3;
    }
  }
  unlock();
}

bool ObjectStore::contains(const std::string& id) {
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), false);
  bool ok = e && e->state == 2;
  unlock();
  return ok;
}

bool ObjectStore::remove(const std::string& id) {
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), false);
  bool ok = e != nullptr && e->state != 4 && e->state != 5;
  if (ok) {
    hdr_->num_objects--;
    if (e->state == 1) {
      e->state = 5;  // unsealed: the creator may still be copying in; freed at its seal/abort
    } else if (e->pins > 0) {
      e->state = 4;  // zombie: freed by the last unpin
    } else {
      free_block(e->offset - sizeof(BlockHdr));
      e->state = 3;
    }
  }
  unlock();
  return ok;
}

bool ObjectStore::abort(const std::string& id) {
  lock();
  ObjectEntry* e = find((const uint8_t*)id.data(), false);
  bool ok = e && (e->state == 1 || e->state == 5);
  if (ok) {
    free_block(e->offset - sizeof(BlockHdr));
    if (e->state == 1) hdr_->num_objects--;
    e->state = 3;
  }
  unlock();
  return ok;
}

std::vector<std::string> ObjectStore::lru_candidates(uint64_t max_count) {
  std::vector<std::pair<uint64_t, std::string>> c;
  lock();
  for (uint64_t i = 0; i < hdr_->table_capacity; ++i) {
    ObjectEntry* e = &table_[i];
    if (e->state == 2 && e->pins == 0)
      c.emplace_back(e->lru, std::string((const char*)e->id, kIdBytes));
  }
  unlock();
  std::sort(c.begin(), c.end());
  std::vector<std::string> out;
  for (size_t i = 0; i < c.size() && i < max_count; ++i) out.push_back(c[i].second);
  return out;
}

std::vector<std::string> ObjectStore::list_ids() {
  std::vector<std::string> out;
  lock();
  for (uint64_t i = 0; i < hdr_->table_capacity; ++i)
    if (table_[i].state == 2) out.emplace_back((const char*)table_[i].id, kIdBytes);
  unlock();
  return out;
}

uint64_t ObjectStore::largest_free() {
  lock();
  uint64_t m = 0;
  for (uint64_t f = hdr_->free_head; f; f = B(f)->next_free) m = std::max(m, B(f)->size);
  unlock();
  return m > sizeof(BlockHdr) ? m - sizeof(BlockHdr) : 0;
}

// Large copies into the arena with non-temporal (streaming) stores: the
// destination lines are never read back by the writer, so regular stores would
// pay a read-for-ownership of every line (twice the memory traffic); glibc only
// switches to streaming stores above ~3/4 of the L3, which a VM reporting a
// 300 MiB L3 never reaches. AVX-512 when the CPU has it, AVX2 otherwise.
__attribute__((target("avx512f"))) static void stream_copy512(uint8_t* d, const uint8_t* s, uint64_t n) {
  for (uint64_t i = 0; i < n; i += 64)
    _mm512_stream_si512((__m512i*)(d + i), _mm512_loadu_si512((const void*)(s + i)));
}
__attribute__((target("avx2"))) static void stream_copy256(uint8_t* d, const uint8_t* s, uint64_t n) {
  for (uint64_t i = 0; i < n; i += 32)
    _mm256_stream_si256((__m256i*)(d + i), _mm256_loadu_si256((const __m256i*)(s + i)));
}
static void big_copy(uint8_t* d, const uint8_t* s, uint64_t n) {
  static const int isa = __builtin_cpu_supports("avx512f") ? 2 : (__builtin_cpu_supports("avx2") ? 1 : 0);
  if (n < (1u << 20) || isa == 0) {
    memcpy(d, s, n);
    return;
  }
  const uint64_t head = (64 - ((uintptr_t)d & 63)) & 63;  // align the destination to a line
  memcpy(d, s, head);
  d += head, s += head, n -= head;
  const uint64_t body = n & ~63ull;
  if (isa == 2) stream_copy512(d, s, body);
  else stream_copy256(d, s, body);
  _mm_sfence();  // streaming stores are weakly ordered: drain before the object is sealed
  memcpy(d + body, s + body, n - body);
}

// Claim up to `want` extra copy threads from the node-wide budget. Returns
// (slot << 16) | threads; threads == 0: nothing claimed. Slots of dead processes are
// reclaimed while summing the active claims; the count is advisory (two claimers may
// both see room and overshoot briefly), which is all a copy-thread budget needs.
uint32_t ObjectStore::claim_copy_threads(uint32_t want, uint32_t budget) {
  uint32_t active = 0;
  int free_slot = -1;
  for (int i = 0; i < Header::kCopyClaims; ++i) {
    uint64_t v = __atomic_load_n(&hdr_->copy_claims[i], __ATOMIC_ACQUIRE);
    if (v == 0) {
      if (free_slot < 0) free_slot = i;
      continue;
    }
    const pid_t pid = (pid_t)(v >> 32);
    if (kill(pid, 0) != 0 && errno == ESRCH) {  // claimant died mid-put: reclaim
      if (__atomic_compare_exchange_n(&hdr_->copy_claims[i], &v, 0ull, false, __ATOMIC_ACQ_REL,
                                      __ATOMIC_RELAXED) && free_slot < 0)
        free_slot = i;
      continue;
    }
    active += (uint32_t)(v & 0xffffffffu);
  }
  if (active >= budget || free_slot < 0) return 0;
  const uint32_t take = std::min(want, budget - active);
  if (take == 0) return 0;
  const uint64_t mine = ((uint64_t)(uint32_t)getpid() << 32) | take;
  for (int i = free_slot; i < Header::kCopyClaims; ++i) {
    uint64_t e = 0;
    if (__atomic_compare_exchange_n(&hdr_->copy_claims[i], &e, mine, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED))
      return ((uint32_t)i << 16) | take;
  }
  return 0;
}

uint32_t ObjectStore::copy_threads_claimed() {
  uint32_t active = 0;
  for (int i = 0; i < Header::kCopyClaims; ++i)
    active += (uint32_t)(__atomic_load_n(&hdr_->copy_claims[i], __ATOMIC_ACQUIRE) & 0xffffffffu);
  return active;
}

void ObjectStore::copy_in(uint64_t off, const void* src, uint64_t n, int threads) {
  uint8_t* dst = base_ + off;
  const uint8_t* s = (const uint8_t*)src;
  const uint64_t kMinChunk = 16ull << 20;
  int want = (int)std::min<uint64_t>((uint64_t)std::max(threads, 1), (n + kMinChunk - 1) / kMinChunk);
  if (want <= 1) {
    big_copy(dst, s, n);
    return;
  }
  // claim extra threads from the node-wide budget (the caller's own thread is free)
  uint32_t budget = __atomic_load_n(&hdr_->copy_threads_budget, __ATOMIC_RELAXED);
  if (budget == 0) budget = 4;
  const uint32_t take = claim_copy_threads((uint32_t)(want - 1), budget);
  const int nt = 1 + (int)(take & 0xffff);
  if (nt <= 1) {
    big_copy(dst, s, n);
    return;
  }
  struct Release {
    uint64_t* slot;
    uint64_t v;
    ~Release() {
      uint64_t e = v;  // our claim, unless a claimer wrongly judged us dead and reclaimed it
      __atomic_compare_exchange_n(slot, &e, 0ull, false, __ATOMIC_ACQ_REL, __ATOMIC_RELAXED);
    }
  } release{&hdr_->copy_claims[take >> 16], ((uint64_t)(uint32_t)getpid() << 32) | (take & 0xffff)};
  const uint64_t chunk = ((n + nt - 1) / nt + 4095) & ~4095ull;
  std::vector<std::thread> ts;
  for (int i = 1; i < nt; ++i) {  // chunk 0 on the calling thread
    const uint64_t b = (uint64_t)i * chunk;
    if (b >= n) break;
    const uint64_t e = std::min(n, b + chunk);
    ts.emplace_back([=] { big_copy(dst + b, s + b, e - b); });
  }
  big_copy(dst, s, std::min(n, chunk));
  for (auto& t : ts) t.join();
}

void ObjectStore::prefault_async(uint64_t max_bytes) {
  uint8_t* lo = base_ + (map_size_ - std::min<uint64_t>(map_size_, capacity()));
  const uint64_t n = std::min<uint64_t>(max_bytes, (uint64_t)(base_ + map_size_ - lo));
  if (prefault_.joinable()) return;
  prefault_ = std::thread([this, lo, n] {
#ifndef MADV_POPULATE_WRITE
#define MADV_POPULATE_WRITE 23
#endif
    const uint64_t step = 64ull << 20;
    for (uint64_t o = 0; o < n && !stop_prefault_.load(std::memory_order_relaxed); o += step) {
      const uint64_t len = std::min(step, n - o);
      if (madvise(lo + o, len, MADV_POPULATE_WRITE) != 0 && errno == EINVAL) {
        // older kernels: fault pages in by touching them (a read-modify-write of
        // one byte per page keeps any data a concurrent put already wrote)
        volatile uint8_t* p = lo + o;
        for (uint64_t q = 0; q < len; q += 4096) __atomic_fetch_add(&p[q], 0, __ATOMIC_RELAXED);
      }
    }
  });
}

}  // namespace caamd_rt
