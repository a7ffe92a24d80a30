// tools/tsan/stress.cpp — host ThreadSanitizer driver for the concurrent parts of libbsgpu's
// C++ host mirror (tools/tsan_host.sh builds both with -fsanitize=thread on the host code).
//
// The reference's threading contract: one goroutine per split.Writer, many Writers at once
// (split/split.go:30-37, fs/dir.go:157-174), and goroutine-safe store Puts (store/mem/mem.go:
// 63-64). Mode "cpu" drives everything that needs no GPU from many threads at once:
//   - store/file's write-behind: 8 write groups putting overlapping blob sets with a tiny
//     pending limit, readers and ListRefs beside them, one poisoned blob whose write fails —
//     its error must reach exactly the groups that put it (bs::FileStore, RefPutter groups);
//   - store/mem: aliased Puts of shared pieces, Seal, Delete, Get and ListRefs at once;
//   - split::Reader (no verify) over a hand-built tree, 8 Readers with random seeks;
//   - bsg::parallel_for (the process-wide copy pool) from 8 callers at once.
// Mode "gpu" (on the MI355X box) adds three engines with early chains on three threads, and
// 8 split::Writers into one MemStore and one FileStore, raw
// bsg_open contexts and verifying Readers, all at once (the pooled contexts and hashers).
// Exit status 0 = every check passed; TSan reports go to stderr (halt_on_error=1 makes a race
// fail the run).
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "../../bs_amd/csrc/host_pool.h"
#include "../../include/bs_split.hpp"

using namespace bs;

static std::atomic<int> g_fail{0};
#define CHECK(c)                                                              \
  do {                                                                        \
    if (!(c)) {                                                               \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #c); \
      g_fail++;                                                               \
    }                                                                         \
  } while (0)

static uint64_t splitmix(uint64_t x) {
  x += 0x9E3779B97F4A7C15ull;
  x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
  x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
  return x ^ (x >> 31);
}

// Blob i: deterministic bytes and a deterministic 32-byte "ref" (the stores trust given refs).
struct TestBlob {
  Ref ref;
  Blob blob;
};
static std::vector<TestBlob> make_blobs(size_t n, uint64_t seed) {
  std::vector<TestBlob> v(n);
  for (size_t i = 0; i < n; ++i) {
    const size_t len = splitmix(seed * 1000003 + i) % 3000;
    std::shared_ptr<uint8_t> b(new uint8_t[len ? len : 1], std::default_delete<uint8_t[]>());
    for (size_t k = 0; k < len; ++k) b.get()[k] = (uint8_t)splitmix(seed + i * 7919 + k);
    v[i].blob = Blob{b, len, 0};
    for (int w = 0; w < 4; ++w) {
      const uint64_t h = splitmix(seed ^ (i * 4 + w) ^ 0xABCDEF);
      std::memcpy(v[i].ref.data() + 8 * w, &h, 8);
    }
  }
  return v;
}

static bool same(const std::vector<uint8_t>& got, const Blob& b) {
  return got.size() == b.size && (b.size == 0 || std::memcmp(got.data(), b.bytes(), b.size) == 0);
}

static void filestore_groups(const std::string& root) {
  FileStore fs(root);
  fs.SetWriteBehindLimit(4096);  // a few blobs pending at most: Puts wait on the writers
  const auto blobs = make_blobs(1200, 11);
  // poison one blob: its directory path (blobs/hh/hhhh) is a regular file, so its write fails
  // (ENOTDIR); it is the first blob no other blob shares that directory with
  size_t poison = 0;
  for (; poison < blobs.size(); ++poison) {
    int same_dir = 0;
    for (const TestBlob& b : blobs) same_dir += b.ref[0] == blobs[poison].ref[0] &&
                                               b.ref[1] == blobs[poison].ref[1];
    if (same_dir == 1) break;
  }
  const std::string path = fs.BlobPath(blobs[poison].ref);
  const std::string dir = path.substr(0, path.find_last_of('/'));
  const std::string parent = dir.substr(0, dir.find_last_of('/'));
  ::mkdir(root.c_str(), 0755);
  ::mkdir((root + "/blobs").c_str(), 0755);
  ::mkdir(parent.c_str(), 0755);
  FILE* f = std::fopen(dir.c_str(), "w");
  CHECK(f != nullptr);
  if (f) std::fclose(f);

  constexpr int kThreads = 8;
  std::vector<std::thread> th;
  std::vector<int> put_poison(kThreads, 0);
  std::atomic<bool> writers_done{false};
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      const uint64_t g = fs.OpenGroup();
      bool saw_error = false;
      std::mt19937_64 rng(t);
      for (int rep = 0; rep < 3; ++rep) {
        for (size_t i = (size_t)t % 3; i < blobs.size(); i += 1 + (size_t)(rng() % 3)) {
          if (i == poison && t % 2) continue;  // even threads only put the poisoned blob
          if (i == poison) put_poison[t] = 1;
          bool added = false;
          Status s = fs.PutBlob(blobs[i].ref, blobs[i].blob, &added, g);
          CHECK(s.ok());
        }
        if (rep == 1) saw_error |= !fs.Flush(g).ok();  // mid-way, as a Writer's node store
      }
      Status s = fs.Flush(g);
      saw_error |= !s.ok();
      // the poisoned blob's failure is reported to exactly the groups that put it
      CHECK(saw_error == (put_poison[t] != 0));
      fs.CloseGroup(g);
    });
  }
  th.emplace_back([&] {  // a reader beside the writers: pending or on disk, always whole
    std::mt19937_64 rng(99);
    while (!writers_done.load()) {
      const size_t i = rng() % blobs.size();
      std::vector<uint8_t> got;
      Status s = fs.Get(blobs[i].ref, &got);
      if (s.ok()) CHECK(same(got, blobs[i].blob));
      Blob b;
      if (fs.GetBlob(blobs[i].ref, &b).ok()) CHECK(b.size == blobs[i].blob.size);
    }
  });
  th.emplace_back([&] {
    while (!writers_done.load()) {
      size_t n = 0;
      (void)fs.ListRefs(Zero, [&](const Ref&) {
        ++n;
        return Status::Ok();
      });
      std::this_thread::sleep_for(std::chrono::milliseconds(5));
    }
  });
  for (int t = 0; t < kThreads; ++t) th[t].join();
  writers_done = true;
  for (size_t t = kThreads; t < th.size(); ++t) th[t].join();
  CHECK(poison < blobs.size());
  // every blob but the poisoned one is on disk, whole
  for (size_t i = 0; i < blobs.size(); ++i) {
    std::vector<uint8_t> got;
    Status s = fs.Get(blobs[i].ref, &got);
    if (i == poison) {
      CHECK(!s.ok());
    } else {
      CHECK(s.ok() && same(got, blobs[i].blob));
    }
  }
}

static void memstore_shares() {
  MemStore ms;
  constexpr int kThreads = 8;
  constexpr size_t kPiece = 1 << 20;
  std::vector<std::thread> th;
  for (int t = 0; t < kThreads; ++t) {
    th.emplace_back([&, t] {
      std::mt19937_64 rng(t + 100);
      for (int p = 0; p < 6; ++p) {
        // a "Write piece" cut into chunks, every chunk an alias of the piece (as split::Writer)
        std::shared_ptr<uint8_t> piece(new uint8_t[kPiece], std::default_delete<uint8_t[]>());
        for (size_t k = 0; k < kPiece; k += 8) {
          const uint64_t v = splitmix((uint64_t)t << 40 | (uint64_t)p << 32 | k);
          std::memcpy(piece.get() + k, &v, 8);
        }
        std::vector<Ref> mine;
        for (size_t off = 0; off < kPiece;) {
          const size_t len = std::min(kPiece - off, (size_t)(1000 + rng() % 60000));
          Ref r;
          for (int w = 0; w < 4; ++w) {
            const uint64_t h =
                splitmix((uint64_t)t << 56 ^ (uint64_t)p << 48 ^ (uint64_t)off << 4 ^ (uint64_t)w);
            std::memcpy(r.data() + 8 * w, &h, 8);
          }
          Blob b{std::shared_ptr<const uint8_t>(piece, piece.get() + off), len, kPiece};
          bool added = false;
          CHECK(ms.PutBlob(r, b, &added).ok() && added);
          mine.push_back(r);
          off += len;
        }
        ms.Seal(Blob{piece, kPiece, 0});
        // delete most of them: the survivors get copied out, the piece is released
        for (size_t k = 0; k < mine.size(); ++k)
          if (k % 5) CHECK(ms.Delete(mine[k]).ok());
        for (size_t k = 0; k < mine.size(); k += 5) {
          std::vector<uint8_t> got;
          CHECK(ms.Get(mine[k], &got).ok());
        }
        size_t n = 0;
        (void)ms.ListRefs(Zero, [&](const Ref&) {
          ++n;
          return Status::Ok();
        });
        (void)ms.HeldBytes();
      }
    });
  }
  for (auto& x : th) x.join();
  // 6 pieces x 8 threads, a fifth of each survives (copied out): far less than 48 MiB held
  CHECK(ms.HeldBytes() < (size_t)kThreads * 6 * kPiece / 2);
}

// A split tree built by hand (no hashing: the stores trust the refs given to PutWithRef): leaf
// nodes of 4 chunks, one root over them.
static void readers_over_tree() {
  MemStore ms;
  std::vector<uint8_t> data(3 << 20);
  for (size_t k = 0; k < data.size(); ++k) data[k] = (uint8_t)splitmix(k);
  split::Node root;
  root.size = data.size();
  uint64_t off = 0;
  int leafno = 0;
  std::mt19937_64 rng(5);
  while (off < data.size()) {
    split::Node leaf;
    leaf.offset = off;
    for (int c = 0; c < 4 && off < data.size(); ++c) {
      const uint64_t len = std::min<uint64_t>(data.size() - off, 20000 + rng() % 90000);
      Ref r{};
      const uint64_t h = splitmix(off + 1);
      std::memcpy(r.data(), &h, 8);
      bool added;
      CHECK(ms.PutWithRef(r, data.data() + off, len, &added).ok());
      leaf.leaves.push_back(split::Child{r, off});
      off += len;
    }
    leaf.size = off - leaf.offset;
    const std::string b = leaf.Marshal();
    Ref lr{};
    const uint64_t h = splitmix(0xF00D + leafno++);
    std::memcpy(lr.data(), &h, 8);
    lr[31] = 1;
    bool added;
    CHECK(ms.PutWithRef(lr, reinterpret_cast<const uint8_t*>(b.data()), b.size(), &added).ok());
    root.nodes.push_back(split::Child{lr, leaf.offset});
  }
  const std::string rb = root.Marshal();
  Ref rr{};
  rr[0] = 0xEE;
  bool added;
  CHECK(ms.PutWithRef(rr, reinterpret_cast<const uint8_t*>(rb.data()), rb.size(), &added).ok());
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) {
    th.emplace_back([&, t] {
      Status err;
      auto rd = split::Reader::New(&ms, rr, &err);
      CHECK(rd != nullptr);
      if (!rd) return;
      std::mt19937_64 r2(t);
      std::vector<uint8_t> buf(200000);
      for (int k = 0; k < 200; ++k) {
        const uint64_t at = r2() % data.size();
        const size_t n = std::min<size_t>(data.size() - at, 1 + r2() % buf.size());
        rd->Seek((int64_t)at, 0);
        size_t got = 0, total = 0;
        bool eof = false;
        while (total < n && !eof) {
          CHECK(rd->Read(buf.data() + total, n - total, &got, &eof).ok());
          total += got;
        }
        CHECK(total == n && std::memcmp(buf.data(), data.data() + at, n) == 0);
      }
    });
  }
  for (auto& x : th) x.join();
}

static void pool_callers() {
  std::vector<std::thread> th;
  for (int t = 0; t < 8; ++t) {
    th.emplace_back([t] {
      for (int rep = 0; rep < 50; ++rep) {
        const size_t n = 1 + (size_t)(t * 7 + rep) % 40;
        std::vector<uint64_t> out(n, 0);
        bsg::parallel_for(n, [&](size_t i) { out[i] = splitmix(i + (uint64_t)t); });
        for (size_t i = 0; i < n; ++i) CHECK(out[i] == splitmix(i + (uint64_t)t));
      }
    });
  }
  for (auto& x : th) x.join();
}

// ---- gpu mode -----------------------------------------------------------------------------
static std::vector<uint8_t> stream_bytes(uint64_t seed, size_t n) {
  std::vector<uint8_t> v(n);
  for (size_t k = 0; k < n; k += 8) {
    const uint64_t w = splitmix(seed * 0x100000000ull + k);
    std::memcpy(v.data() + k, &w, std::min<size_t>(8, n - k));
  }
  return v;
}

static Ref write_stream(Store* st, const std::vector<uint8_t>& d, const split::Options& o,
                        size_t piece) {
  Status err;
  auto w = split::Writer::New(st, o, &err);
  CHECK(w != nullptr);
  if (!w) return Ref{};
  for (size_t i = 0; i < d.size(); i += piece)
    CHECK(w->Write(d.data() + i, std::min(piece, d.size() - i)).ok());
  CHECK(w->Close().ok());
  return w->Root();
}

static void gpu_writers(const std::string& root) {
  const size_t MiB = 1 << 20;
  struct Job {
    uint64_t seed;
    size_t n;
    unsigned bits;
    int min_size;
    unsigned fanout;
    size_t piece;
  };
  const std::vector<Job> jobs = {{1, 24 * MiB, 16, 1024, 8, 32 << 10}, {2, 40 * MiB, 13, 64, 4, 32 * MiB},
                                 {3, 17 * MiB, 12, 256, 2, 32 << 10}, {4, 33 * MiB, 20, 4096, 8, 32 * MiB},
                                 {1, 24 * MiB, 16, 1024, 8, 32 * MiB}, {5, 9 * MiB, 10, 17, 3, 32 << 10},
                                 {3, 17 * MiB, 12, 256, 2, 32 * MiB}, {6, 28 * MiB, 16, 1024, 8, 32 << 10}};
  std::vector<std::vector<uint8_t>> data;
  for (const Job& j : jobs) data.push_back(stream_bytes(j.seed, j.n));
  for (int pass = 0; pass < 2; ++pass) {
    MemStore ms;
    FileStore fs(root + "/gpu" + std::to_string(pass));
    fs.SetWriteBehindLimit(1 << 20);
    Store* st = pass == 0 ? static_cast<Store*>(&ms) : static_cast<Store*>(&fs);
    std::vector<Ref> roots(jobs.size());
    std::vector<std::thread> th;
    for (size_t i = 0; i < jobs.size(); ++i)
      th.emplace_back([&, i] {
        split::Options o;
        o.bits = jobs[i].bits;
        o.min_size = jobs[i].min_size;
        o.fanout = jobs[i].fanout;
        roots[i] = write_stream(st, data[i], o, jobs[i].piece);
      });
    // a raw streaming context and a hasher beside the Writers
    th.emplace_back([&] {
      int rc = 0;
      bsg_params p = bsg_params_default();
      bsg_ctx* c = bsg_open(0, &p, nullptr, &rc);
      CHECK(c != nullptr);
      if (!c) return;
      CHECK(bsg_write(c, data[0].data(), data[0].size()) == BSG_OK);
      CHECK(bsg_close(c) == BSG_OK);
      std::vector<bsg_chunk> out(bsg_pending(c));
      const size_t got = bsg_drain(c, out.data(), out.size());
      uint64_t total = 0;
      for (size_t k = 0; k < got; ++k) total += out[k].len;
      CHECK(total == data[0].size());
      bsg_free(c);
    });
    for (auto& x : th) x.join();
    CHECK(roots[0] == roots[4] && roots[2] == roots[6]);
    // verifying Readers, concurrently
    std::vector<std::thread> rd;
    for (size_t i = 0; i < jobs.size(); ++i)
      rd.emplace_back([&, i] {
        Status err;
        auto r = split::Reader::New(st, roots[i], &err, true, 0);
        CHECK(r != nullptr);
        if (!r) return;
        std::vector<uint8_t> out(data[i].size());
        size_t total = 0, got = 0;
        bool eof = false;
        while (!eof && total < out.size()) {
          CHECK(r->Read(out.data() + total, std::min<size_t>(MiB, out.size() - total), &got, &eof).ok());
          total += got;
          if (!got) break;
        }
        CHECK(total == out.size() && out == data[i]);
      });
    for (auto& x : rd) x.join();
  }
}

// Three engines on three threads, each a 272 MiB device-resident run twice, so the early chains
// (a second stream, cross-stream events) run beside each other; every run's records must equal
// the same engine's run with the early chains off.
static void gpu_engines() {
  const uint64_t n = 272ull << 20;
  std::vector<std::thread> th;
  for (int t = 0; t < 3; ++t)
    th.emplace_back([t, n] {
      int rc = 0;
      bsg_engine* e = bsg_engine_create(0, nullptr, &rc);
      CHECK(e != nullptr);
      if (!e) return;
      uint8_t* d = static_cast<uint8_t*>(bsg_device_malloc(0, n + BSG_READ_SLACK));
      CHECK(d != nullptr);
      if (!d) {
        bsg_engine_destroy(e);
        return;
      }
      CHECK(bsg_fill_splitmix(0, d, n, 0x7A5 + t, bsg_engine_stream(e)) == BSG_OK);
      const uint64_t off = 0, len = n;
      bsg_params p = bsg_params_default();
      std::vector<bsg_chunk> first;
      for (int rep = 0; rep < 3; ++rep) {
        CHECK(bsg_engine_run(e, d, &off, &len, 1, &p) == BSG_OK);
        uint64_t m = 0;
        CHECK(bsg_engine_finish(e, &m) == BSG_OK);
        std::vector<bsg_chunk> out(m);
        CHECK(bsg_engine_copy_chunks(e, out.data(), m) == BSG_OK);
        if (rep == 0) {
          first = out;
        } else {
          CHECK(out.size() == first.size() &&
                std::memcmp(out.data(), first.data(), out.size() * sizeof(bsg_chunk)) == 0);
        }
      }
      bsg_device_free(0, d);
      bsg_engine_destroy(e);
    });
  for (auto& x : th) x.join();
}

int main(int argc, char** argv) {
  const std::string mode = argc > 1 ? argv[1] : "cpu";
  char tmpl[] = "/tmp/bsg_tsan_XXXXXX";
  const char* dir = ::mkdtemp(tmpl);
  if (!dir) return 2;
  const std::string root = dir;
  if (mode == "cpu" || mode == "all") {
    filestore_groups(root + "/fs");
    std::fprintf(stderr, "filestore_groups done\n");
    memstore_shares();
    std::fprintf(stderr, "memstore_shares done\n");
    readers_over_tree();
    std::fprintf(stderr, "readers_over_tree done\n");
    pool_callers();
    std::fprintf(stderr, "pool_callers done\n");
  }
  if (mode == "gpu" || mode == "all") {
    gpu_writers(root);
    std::fprintf(stderr, "gpu_writers done\n");
    gpu_engines();
    std::fprintf(stderr, "gpu_engines done\n");
  }
  std::string rm = "rm -rf " + root;
  (void)std::system(rm.c_str());
  std::printf("%s: %s (%d failed checks)\n", mode.c_str(), g_fail ? "FAIL" : "ok", g_fail.load());
  return g_fail ? 1 : 0;
}
