// Concurrency stress of the native runtime for sanitizer builds (SURVEY §5 race
// detection; reference: Ray's TSAN/ASAN CI builds of src/ray). Built and run by
// tests/test_native_sanitizers.py with -fsanitize=thread and, separately,
// -fsanitize=address,undefined:
//
//  * object store: T threads x 2 processes (fork) hammer one shm arena with
//    create / copy / seal / lookup+pin / unpin / remove / abort, including the
//    remove-while-unsealed and remove-while-pinned paths, and verify every payload
//    they read back;
//  * channel: one writer, R readers through the shm ring with checksummed
//    messages, exercising wrap-around and reader back-pressure.
//
// Exit code 0 = all checks passed (the sanitizers abort on their own findings).
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "channel.h"
#include "object_store.h"

using namespace caamd_rt;

static std::string oid(int proc, int t, int i) {
  char b[24];
  memset(b, 0, sizeof(b));
  snprintf(b, sizeof(b), "p%d-t%d-i%d", proc, t, i);
  return std::string(b, 24);
}

static int store_worker(const std::string& name, int proc, int threads, int iters) {
  ObjectStore st(name, 0, 0, false);
  std::atomic<int> bad{0};
  std::vector<std::thread> ts;
  for (int t = 0; t < threads; ++t) {
    ts.emplace_back([&, t] {
      for (int i = 0; i < iters; ++i) {
        const std::string id = oid(proc, t, i);
        const uint64_t n = 64 + (uint64_t)((i * 2654435761u + t) % 8192);
        const int64_t off = st.create(id, n, (uint64_t)i);
        if (off < 0) continue;  // full: fine under pressure
        if (i % 17 == 0) {      // removed while the creator is still writing
          st.remove(id);
        }
        uint8_t* p = st.base() + off;
        for (uint64_t k = 0; k < n; ++k) p[k] = (uint8_t)(k + i + t);
        if (i % 29 == 0) {
          st.abort(id);
          continue;
        }
        st.seal(id);
        uint64_t o2, sz, meta;
        if (st.lookup(id, &o2, &sz, &meta, true)) {
          const uint8_t* q = st.base() + o2;
          for (uint64_t k = 0; k < sz; k += 97)
            if (q[k] != (uint8_t)(k + i + t)) bad++;
          if (i % 5 == 0) st.remove(id);  // remove while pinned (zombie until unpin)
          st.unpin(id);
        }
        if (i % 3 == 0) st.remove(id);
        // look at a neighbour's objects too (cross-thread reads)
        const std::string other = oid(proc, (t + 1) % threads, i > 0 ? i - 1 : 0);
        if (st.lookup(other, &o2, &sz, &meta, true)) {
          volatile uint8_t s = st.base()[o2];
          (void)s;
          st.unpin(other);
        }
      }
    });
  }
  for (auto& th : ts) th.join();
  // clean up everything this process created
  for (int t = 0; t < threads; ++t)
    for (int i = 0; i < iters; ++i) st.remove(oid(proc, t, i));
  if (bad) fprintf(stderr, "store proc %d: %d corrupted reads\n", proc, bad.load());
  return bad ? 1 : 0;
}

static int channel_test(const std::string& name, int readers, int msgs) {
  Channel w(name, true, readers, 3, 4096);
  std::atomic<int> bad{0};
  std::vector<std::thread> rs;
  for (int r = 0; r < readers; ++r) {
    rs.emplace_back([&, r] {
      Channel c(name, false, readers, 3, 4096);
      std::vector<uint8_t> buf(4096);
      for (int m = 0; m < msgs; ++m) {
        uint64_t len = 0, flags = 0;
        const uint8_t* data = nullptr;
        int rc = c.begin_read(r, &data, &len, &flags, 30.0);
        if (rc != 0) {
          bad++;
          return;
        }
        uint32_t sum = 0;
        for (uint64_t k = 4; k < len; ++k) sum += data[k];
        uint32_t want;
        memcpy(&want, data, 4);
        if (sum != want || flags != (uint64_t)m) bad++;
        c.end_read(r);
      }
    });
  }
  std::vector<uint8_t> msg(4096);
  for (int m = 0; m < msgs; ++m) {
    const uint64_t len = 8 + (uint64_t)((m * 7919) % 4000);
    uint32_t sum = 0;
    for (uint64_t k = 4; k < len; ++k) {
      msg[k] = (uint8_t)(m + k);
      sum += msg[k];
    }
    memcpy(msg.data(), &sum, 4);
    if (w.write(msg.data(), len, (uint64_t)m, 30.0) != 0) bad++;
  }
  for (auto& t : rs) t.join();
  w.unlink();
  if (bad) fprintf(stderr, "channel: %d bad messages\n", bad.load());
  return bad ? 1 : 0;
}

#ifdef STRESS_CANARY_RACE
// deliberately racy: proves the ThreadSanitizer build reports races at all
static int canary_counter = 0;
static void canary() {
  std::thread a([] { for (int i = 0; i < 100000; ++i) canary_counter++; });
  std::thread b([] { for (int i = 0; i < 100000; ++i) canary_counter++; });
  a.join();
  b.join();
  printf("canary %d\n", canary_counter);
}
#endif

int main(int argc, char** argv) {
#ifdef STRESS_CANARY_RACE
  canary();
  return 0;
#endif
  const int threads = argc > 1 ? atoi(argv[1]) : 4;
  const int iters = argc > 2 ? atoi(argv[2]) : 2000;
  const std::string sname = "/caamd_stress_" + std::to_string(getpid());
  int rc = 0;
  {
    ObjectStore owner(sname, 32u << 20, 1 << 14, true);
    const int procs = 2;
    std::vector<pid_t> kids;
    for (int p = 1; p < procs; ++p) {
      pid_t k = fork();
      if (k == 0) _exit(store_worker(sname, p, threads, iters));
      kids.push_back(k);
    }
    rc |= store_worker(sname, 0, threads, iters);
    for (pid_t k : kids) {
      int status = 0;
      waitpid(k, &status, 0);
      if (!WIFEXITED(status) || WEXITSTATUS(status) != 0) rc |= 2;
    }
    if (owner.num_objects() != 0) {
      fprintf(stderr, "store: %llu objects leaked\n", (unsigned long long)owner.num_objects());
      rc |= 4;
    }
    owner.unlink();
  }
  rc |= channel_test("/caamd_stress_ch_" + std::to_string(getpid()), 3, 3000) ? 8 : 0;
  printf("stress_runtime rc=%d\n", rc);
  return rc;
}
