// bs_split.hpp — C++ host mirror of the reference's split package and Store surface, built on
// libbsgpu's C ABI (include/bsgpu.h). Same names, argument meaning and error behaviour as the
// Go originals; the per-byte chunking and every SHA-256 run on the GPU.
//
//   bs::Ref / bs::Zero / RefString        bs.go:12-36
//   bs::Store (Get / Put / ListRefs)       store.go:9-42
//   bs::RefPutter (optional, like MultiPutter store.go:44-47): Put with a ref the caller already
//                 computed on the GPU, so a backend need not hash the blob again
//   bs::MemStore                           store/mem/mem.go:17-124
//   bs::FileStore                          store/file/file.go:20-154 (blob layout and ListRefs;
//                                          anchors are out of scope)
//   bs::split::Writer  New/Write/Close/Root, options Bits/MinSize/Fanout   split/split.go:30-165
//   bs::split::Reader  New/Read/Seek/Size                                  split/split.go:173-303
//   bs::split::Node / Child (proto3 wire format)                           split/split.proto:6-26
#pragma once

#include <array>
#include <condition_variable>
#include <deque>
#include <cstddef>
#include <cstdint>
#include <functional>
#include <future>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "bsgpu.h"

namespace bs {

using Ref = std::array<uint8_t, 32>;
extern const Ref Zero;  // bs.Zero
std::string RefString(const Ref& r);  // lowercase hex (bs.go:29-31)
inline bool RefLess(const Ref& a, const Ref& b) { return a < b; }  // bs.go:34-36

// Go `error` -> Status: code 0 is nil; other codes are BSG_* (bsgpu.h) or kNotFound.
struct Status {
  int code = 0;
  std::string msg;
  bool ok() const { return code == 0; }
  static Status Ok() { return Status{}; }
  static Status Err(int c, std::string m) { return Status{c, std::move(m)}; }
};
constexpr int kNotFound = BSG_ENOTFOUND;  // bs.ErrNotFound (store.go:63)
constexpr int kCorrupt = BSG_ECORRUPT;    // a fetched blob does not hash to its ref (Reader verify)
constexpr int kIO = BSG_EIO;              // filesystem error (errno text in Status::msg)

struct Blob;

class Store {
 public:
  virtual ~Store() = default;
  virtual Status Get(const Ref& ref, std::vector<uint8_t>* out) = 0;
  // Get with shared ownership of the bytes: a store holding blobs in memory hands out its own
  // (store/mem), others read into a new buffer. The bytes never change afterwards.
  virtual Status GetBlob(const Ref& ref, Blob* out);
  // Put adds the blob if absent; *ref = its SHA-256, *added = whether it was new.
  virtual Status Put(const uint8_t* data, size_t n, Ref* ref, bool* added) = 0;
  // Calls f for each ref > start in lexicographic order (store.go:21-23).
  virtual Status ListRefs(const Ref& start, const std::function<Status(const Ref&)>& f) = 0;
};

// A blob's bytes with shared ownership: `data` points into memory kept alive by the
// shared_ptr (an aliasing pointer into a larger buffer, e.g. a Writer's input piece), so a store
// can retain a chunk without copying it, as store/mem retains the caller's slice
// (store/mem/mem.go:71). The bytes must never change afterwards.
struct Blob {
  std::shared_ptr<const uint8_t> data;
  size_t size = 0;
  // bytes of the buffer `data` aliases into when that buffer is larger than the blob (a Write
  // piece); 0 when the blob owns exactly its bytes
  size_t base_size = 0;
  const uint8_t* bytes() const { return data.get(); }
};

// Write groups: a store that writes behind (store/file) accepts a blob before it is durable.
// Each caller (one split::Writer) opens a group, puts its blobs in it, and Flush(group) waits for
// exactly the blobs that group put — including ones another group had already queued when this
// one asked for them — and returns the first error among them (then forgets it). So one
// Writer's failed write is reported to that Writer only, and a Writer can guarantee "a tree node
// is stored only after every blob under it is" (split/split.go:71-77,118 store chunks before
// their node) by flushing its group before it stores a node. Group 0 is the ungrouped caller.
class RefPutter {
 public:
  virtual ~RefPutter() = default;
  virtual Status PutWithRef(const Ref& ref, const uint8_t* data, size_t n, bool* added) = 0;
  // The same with shared ownership of the bytes: a store that retains blobs in memory keeps
  // the Blob itself (no copy); others just read it.
  virtual Status PutBlob(const Ref& ref, const Blob& b, bool* added, uint64_t group = 0) {
    (void)group;
    return PutWithRef(ref, b.bytes(), b.size, added);
  }
  virtual uint64_t OpenGroup() { return 0; }
  virtual void CloseGroup(uint64_t group) { (void)group; }
  // Waits for the group's accepted-but-unwritten blobs; the first error among them.
  virtual Status Flush(uint64_t group) {
    (void)group;
    return Status::Ok();
  }
  // No more blobs aliasing `whole`'s buffer will be put (split::Writer: a Write piece whose
  // bytes are all emitted as chunks). A store that keeps such aliases (store/mem) then keeps
  // private copies of them instead, if they hold less than half of the buffer alive.
  virtual void Seal(const Blob& whole) { (void)whole; }
};

// Batched/one-off SHA-256 of host bytes on the GPU (bsg_hasher: persistent device buffers +
// stream, created on first use).
class GpuHasher {
 public:
  explicit GpuHasher(int device = 0) : device_(device) {}
  ~GpuHasher();
  GpuHasher(const GpuHasher&) = delete;
  GpuHasher& operator=(const GpuHasher&) = delete;
  Status Sum(const uint8_t* data, size_t n, Ref* out);
  // refs[i] = SHA-256 of base[off[i] .. off[i] + len[i]) for n blobs, one GPU call.
  Status SumBatch(const uint8_t* base, const uint64_t* off, const uint64_t* len, size_t n,
                  Ref* refs);
  // refs[i] = SHA-256 of ptrs[i][0 .. len[i]) (scattered blobs), one GPU call.
  Status SumPtrs(const uint8_t* const* ptrs, const uint64_t* len, size_t n, Ref* refs);

 private:
  int device_;
  std::mutex mu_;
  bsg_hasher* h_ = nullptr;
};

class MemStore : public Store, public RefPutter {
 public:
  explicit MemStore(int device = 0) : hasher_(device) {}
  Status Get(const Ref& ref, std::vector<uint8_t>* out) override;
  Status GetBlob(const Ref& ref, Blob* out) override;  // the stored Blob itself, no copy
  Status Put(const uint8_t* data, size_t n, Ref* ref, bool* added) override;
  Status ListRefs(const Ref& start, const std::function<Status(const Ref&)>& f) override;
  Status PutWithRef(const Ref& ref, const uint8_t* data, size_t n, bool* added) override;
  // Keeps b itself (mem.go:71 keeps the caller's slice): no copy of the chunk bytes.
  Status PutBlob(const Ref& ref, const Blob& b, bool* added, uint64_t group = 0) override;
  void Seal(const Blob& whole) override;
  // bs.DeleterStore (store.go:50-54): removes ref if present; absent refs are not an error
  // (mem.go:79-85). When the blobs left aliasing a sealed buffer hold less than half of it,
  // they are copied out, so deleting most of a Write's chunks frees the Write's memory.
  Status Delete(const Ref& ref);
  size_t Size() const;
  // Bytes of the buffers the store keeps alive (its own copies plus every aliased buffer
  // once), for tests and diagnostics.
  size_t HeldBytes() const;

 private:
  // Blobs aliasing one larger buffer (keyed by the buffer's owner): how much of it is live.
  struct Share {
    size_t base_size = 0, live = 0;
    bool sealed = false;
    std::vector<Ref> refs;
  };
  using Owner = std::weak_ptr<const uint8_t>;
  void MaybeCompact(std::map<Owner, Share, std::owner_less<Owner>>::iterator it);  // under mu_
  mutable std::mutex mu_;
  std::map<Ref, Blob> blobs_;
  std::map<Owner, Share, std::owner_less<Owner>> shares_;
  GpuHasher hasher_;
};

// store/file: blobs live at <root>/blobs/<hex[:2]>/<hex[:4]>/<hex> (file.go:33-40). Put hashes
// on the GPU and creates the file with O_CREAT|O_EXCL (an existing file means "already
// present", file.go:52-76); PutWithRef skips the hash when the caller has the GPU's ref.
class FileStore : public Store, public RefPutter {
 public:
  explicit FileStore(std::string root, int device = 0)
      : root_(std::move(root)), hasher_(device) {}
  ~FileStore() override;
  Status Get(const Ref& ref, std::vector<uint8_t>* out) override;
  Status GetBlob(const Ref& ref, Blob* out) override;
  Status Put(const uint8_t* data, size_t n, Ref* ref, bool* added) override;
  Status ListRefs(const Ref& start, const std::function<Status(const Ref&)>& f) override;
  Status PutWithRef(const Ref& ref, const uint8_t* data, size_t n, bool* added) override;
  // Write-behind (split.Writer's chunks): the Blob is kept, and written by a pool of writer
  // threads; Get sees it at once, Flush(group) waits for the group's files. *added: not already
  // pending (a blob pending for another group is shared: this group's Flush waits for it too).
  Status PutBlob(const Ref& ref, const Blob& b, bool* added, uint64_t group = 0) override;
  uint64_t OpenGroup() override;
  void CloseGroup(uint64_t group) override;
  Status Flush(uint64_t group) override;
  // Waits for every pending blob (ListRefs, the destructor); the ungrouped callers' first error.
  Status FlushAll();
  std::string BlobPath(const Ref& ref) const;
  const std::string& Root() const { return root_; }
  // At most this many bytes are pending before PutBlob waits (tests shrink it).
  void SetWriteBehindLimit(uint64_t bytes);

 private:
  Status MkdirFor(const std::string& path);  // os.MkdirAll of the blob's directory, cached
  void Worker();
  std::string root_;
  GpuHasher hasher_;
  std::mutex dir_mu_;
  std::vector<bool> dirs_made_ = std::vector<bool>(1 << 16);  // blobs/hh/hhhh made, by hhhh
  struct Pending {
    Blob blob;
    std::vector<uint64_t> groups;  // every group whose Flush must wait for this write
  };
  struct Group {
    uint64_t outstanding = 0;  // blobs of this group not yet written
    Status err;                // first failed write of the group, until Flush reports it
    bool closed = false;       // CloseGroup called: forget it once outstanding reaches 0
  };
  void Attach(Pending& p, uint64_t group);  // under wb_mu_
  std::mutex wb_mu_;
  std::condition_variable wb_cv_, wb_done_cv_;
  std::deque<Ref> wb_queue_;           // refs of wb_pending_ in arrival order
  std::map<Ref, Pending> wb_pending_;  // accepted, not yet written
  std::map<uint64_t, Group> groups_ = {{0, Group{}}};  // group 0: ungrouped callers
  uint64_t next_group_ = 1;
  uint64_t wb_bytes_ = 0;              // bytes of wb_pending_ (bounded: wb_limit_)
  uint64_t wb_limit_ = 1ull << 30;
  bool wb_stop_ = false;
  std::vector<std::thread> wb_threads_;
  static constexpr int kWriterThreads = 8;
};

bool RefFromHex(const std::string& hex, Ref* out);  // bs.RefFromHex (bs.go)

namespace split {

struct Child {  // split.proto Child {bytes ref = 1; uint64 offset = 2;}
  Ref ref{};
  uint64_t offset = 0;
};
struct Node {  // split.proto Node {nodes = 1; leaves = 2; offset = 3; size = 4;}
  std::vector<Child> nodes, leaves;
  uint64_t offset = 0, size = 0;
  std::string Marshal() const;                    // deterministic proto3, as Go proto.Marshal
  bool Unmarshal(const uint8_t* p, size_t n);
};

// split.Option values (split/split.go:128-165).
struct Options {
  unsigned bits = 16;     // Bits(n)
  int min_size = 1024;    // MinSize(n)
  unsigned fanout = 8;    // Fanout(n)
  int device = 0;         // HIP device that runs the chunker and the hashes
  size_t tile = 0;        // staging tile in bytes (0: library default, 256 MiB)
};
inline Options Bits(Options o, unsigned n) { o.bits = n; return o; }
inline Options MinSize(Options o, int n) { o.min_size = n; return o; }
inline Options Fanout(Options o, unsigned n) { o.fanout = n; return o; }

class Writer {
 public:
  // split.NewWriter(ctx, st, opts...). The store must outlive the Writer.
  static std::unique_ptr<Writer> New(Store* st, const Options& opt, Status* err);
  ~Writer();
  // io.Writer: consumes all of p (copied); chunks found so far are Put to the store.
  Status Write(const uint8_t* p, size_t n, size_t* written = nullptr);
  // Flushes the final chunk, builds the tree root; Root() is valid afterwards. Idempotent.
  Status Close();
  const Ref& Root() const { return root_; }
  // Tests: the stream's first byte has stream offset `base` on the device (bsg_set_stream_base),
  // so that offsets past 2^40 are exercised without writing 1 TiB. Before the first Write; the
  // tree (offsets from 0, as split.Writer's) is unchanged.
  Status SetStreamBase(uint64_t base);

  struct TBNode;
  struct Wrapped;

 private:
  explicit Writer(int device);
  Status Drain();                                   // take and process, on this thread
  size_t TakeRecords(std::vector<bsg_chunk>* out);  // completed chunk records from the context
  Status Process(const std::vector<bsg_chunk>& recs);  // Put + TreeBuilder.Add, stream order
  // A Write's records are processed on a background thread while the Write copies its bytes
  // (the copy waits on the H2D copies; processing is host bookkeeping): Submit hands records
  // over, Join waits for them and returns the first error.
  struct Bg;
  std::unique_ptr<Bg> bg_;
  void Submit(std::vector<bsg_chunk>* recs);
  Status Join();
  Status Add(const Ref& ref, uint64_t len, unsigned level);  // hashsplit TreeBuilder.Add
  Status F(TBNode& n, std::shared_ptr<Wrapped>* out);        // split.go:52-81
  Status PutProto(const Node& node, Ref* ref);               // proto.go:22-29
  // PutProto of several nodes: one batched GPU hash when the store takes refs (RefPutter).
  Status PutProtos(const std::vector<const Node*>& nodes, std::vector<Ref>* refs);
  GpuHasher hasher_;

  Store* st_ = nullptr;
  RefPutter* rp_ = nullptr;
  uint64_t group_ = 0;  // this Writer's write group in rp_ (RefPutter::OpenGroup)
  Options opt_;
  bsg_ctx* ctx_ = nullptr;
  // Stream bytes not yet emitted as chunks, kept as the Write() pieces they arrived in: a
  // piece is dropped once every byte of it is in an emitted chunk, so nothing is ever moved.
  // Chunks inside one piece are handed to the store as aliases of it (Blob), so the piece
  // lives on in the store for as long as a chunk of it does.
  struct Piece {
    std::shared_ptr<uint8_t> buf;
    size_t size = 0;
  };
  std::deque<Piece> pieces_;
  Status Copy(const uint8_t* p, size_t n, uint8_t* dst);  // into dst and pinned staging
  uint64_t base_ = 0;          // stream offset of pieces_.front()[0]
  uint64_t end_ = 0;           // stream offset one past the last byte written
  uint64_t emitted_ = 0;       // stream offset of the next chunk to emit

  std::vector<std::unique_ptr<TBNode>> levels_;
  std::vector<bsg_chunk> drained_;
  Ref root_{};
  bool closed_ = false;
  Status sticky_;
  // where a Writer's time goes (seconds), printed when it is destroyed if BSG_DEBUG_WRITER is set
  // (drain: records processed on the background thread, overlapping the copies; join: what the
  // Writes waited for it)
  struct Timing {
    double copy = 0, drain = 0, join = 0, hash = 0, close = 0, close_dev = 0;
    uint64_t hash_calls = 0;
  } tm_;

 public:
  // tm_ in seconds: [0] Write copies, [1] records processed on the background thread (Put +
  // TreeBuilder.Add, overlapping the copies), [2] Writes and Close waiting for that thread,
  // [3] tree-node hashes (GPU), [4] Close, [5] of which waiting for the last tiles on the device,
  // [6] tree-node hash calls
  void Timings(double out[7]) const {
    out[0] = tm_.copy;
    out[1] = tm_.drain;
    out[2] = tm_.join;
    out[3] = tm_.hash;
    out[4] = tm_.close;
    out[5] = tm_.close_dev;
    out[6] = (double)tm_.hash_calls;
  }
};

// split.Protect (split/split.go:306-322), the gc.ProtectFunc for split trees: the children of
// the Node stored at ref, tree nodes first (each to be traversed the same way), then leaves
// (chunks, not traversed).
struct ProtectPair {
  Ref ref{};
  bool traverse = false;  // true: a child Node (ProtectPair.F = Protect); false: a leaf
};
Status Protect(Store* g, const Ref& ref, std::vector<ProtectPair>* out);

class Reader {
 public:
  // split.NewReader(ctx, g, ref). verify (not in the reference, which trusts its store): the
  // chunks are fetched a window at a time (the leaf nodes from the one being read on, up to
  // kVerifyWindow bytes) and their SHA-256 checked against their refs in one batched GPU call;
  // reads are served from the verified copies, and a mismatch fails the Read with kCorrupt.
  static std::unique_ptr<Reader> New(Store* g, const Ref& root, Status* err,
                                     bool verify = false, int device = 0);
  // io.Reader: returns bytes read; 0 with *eof = true at the end.
  Status Read(uint8_t* buf, size_t n, size_t* got, bool* eof);
  // io.Seeker (whence: 0 start, 1 current, 2 end).
  uint64_t Seek(int64_t offset, int whence);
  uint64_t Size() const { return stack_.front().size; }
  // Verify mode diagnostics: [0] windows verified on the reading thread, [1] windows taken from
  // the background read-ahead, [2] bytes verified, [3] windows started ahead and dropped.
  void Stats(uint64_t out[4]) const {
    out[0] = tm_.sync_windows;
    out[1] = tm_.ahead_windows;
    out[2] = tm_.bytes;
    out[3] = tm_.dropped;
  }

 private:
  Reader() = default;
  static constexpr uint64_t kVerifyWindow = 256ull << 20;  // bytes verified per GPU call
  uint64_t window_bytes_ = kVerifyWindow;                 // (BSG_VERIFY_WINDOW overrides)
  // Verify mode. A resumable walk over the tree's leaf nodes in order (one frame per internal
  // node on the path: the node and its next child), and a window: the verified chunks of a run
  // of leaf nodes, by leaf-node offset, with the walk positioned after them.
  struct Frame {
    Node node;
    size_t next = 0;
  };
  struct Window {
    std::map<uint64_t, std::vector<Blob>> leaves;
    std::vector<Frame> cursor;
    std::vector<uint64_t> covered;  // its leaf-node offsets (also when verification failed)
    Status st;
    bool end = false;               // the walk reached the last leaf node
    double t_walk = 0, t_fetch = 0, t_hash = 0;  // seconds in VerifyRun's phases
    uint64_t bytes = 0;
  };
  Status NextLeafNode(std::vector<Frame>* cur, Node* out, bool* done);
  Window VerifyRun(std::vector<Frame> cur, const Node* first, uint64_t budget);
  Status TakeLeaf();  // cache_ = the verified chunks of stack_.back()
  Store* g_ = nullptr;
  uint64_t pos_ = 0;
  std::vector<Node> stack_;  // stack_[0] is the root
  bool verify_ = false;
  int device_ = 0;
  bool cache_valid_ = false;  // cache_ holds stack_.back()'s leaves
  uint64_t next_leaf_ = 0;    // offset right after the last leaf node taken (verify mode)
  std::vector<Blob> cache_;   // verified chunks of that leaf node
  // verified chunks of the window's later leaf nodes, by leaf-node offset
  std::map<uint64_t, std::vector<Blob>> window_;
  std::unique_ptr<GpuHasher> hasher_;
  // the next window, fetched and verified on a background thread while this one is read
  std::future<Window> ahead_;
  bool ahead_stale_ = false;  // ahead_ was started before a seek: never taken, only dropped
  // where a verifying Reader's time goes (seconds), printed when it is destroyed if
  // BSG_DEBUG_READER is set: windows verified on the reading thread / ahead, VerifyRun's phases
  // summed over all windows, and what reads waited for the window verified ahead
  struct Timing {
    double walk = 0, fetch = 0, hash = 0, wait = 0, sync = 0;
    uint64_t sync_windows = 0, ahead_windows = 0, bytes = 0, dropped = 0;
  } tm_;

 public:
  ~Reader();
};

}  // namespace split
}  // namespace bs
