// bs_split.cpp — C++ host mirror of split.Writer / split.Reader / store/mem over libbsgpu
// (include/bs_split.hpp), plus the C ABI wrappers the Python tests drive (bsg_memstore_*,
// bsg_writer_*, bsg_reader_*).
//
// Tree assembly restates hashsplit v1.1.1's TreeBuilder as wired by split.NewWriter
// (split/split.go:51-90): every chunk is Added with level/fanout; a level-i node closes when a
// chunk of level > i arrives; F turns a finished TreeBuilderNode into a split.Node whose child
// nodes are PutProto'd and whose chunks are Put. Root() folds the open levels and prunes
// single-child roots. Parity of Root with Go is unpinned (the module's source is not in the
// reference tree), chunk boundaries and refs are pinned by the tests.
#include <sys/mman.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <thread>
#include <tuple>

#include "../../include/bs_split.hpp"
#include "host_pool.h"

namespace bs {

const Ref Zero{};

std::string RefString(const Ref& r) {
  static const char* hx = "0123456789abcdef";
  std::string s(64, '0');
  for (int i = 0; i < 32; ++i) {
    s[2 * i] = hx[r[i] >> 4];
    s[2 * i + 1] = hx[r[i] & 15];
  }
  return s;
}

// GpuHashers take their bsg_hasher (device buffers, pinned staging, an engine) from a small
// process-wide pool and give it back when destroyed, so a Reader or store created per file
// does not set one up each time.
namespace {
std::mutex g_hasher_mu;
std::vector<bsg_hasher*>& hasher_pool(int device) {
  static auto* pools = new std::map<int, std::vector<bsg_hasher*>>();  // never destroyed
  return (*pools)[device];
}
bsg_hasher* hasher_acquire(int device) {
  {
    std::lock_guard<std::mutex> g(g_hasher_mu);
    auto& v = hasher_pool(device);
    if (!v.empty()) {
      bsg_hasher* h = v.back();
      v.pop_back();
      return h;
    }
  }
  return bsg_hasher_new(device);
}
void hasher_release(int device, bsg_hasher* h) {
  if (!h) return;
  {
    std::lock_guard<std::mutex> g(g_hasher_mu);
    auto& v = hasher_pool(device);
    if (v.size() < 4) {
      v.push_back(h);
      return;
    }
  }
  bsg_hasher_free(h);
}
}  // namespace

GpuHasher::~GpuHasher() { hasher_release(device_, h_); }

Status Store::GetBlob(const Ref& ref, Blob* out) {
  auto v = std::make_shared<std::vector<uint8_t>>();
  Status s = Get(ref, v.get());
  if (!s.ok()) return s;
  out->size = v->size();
  out->data = std::shared_ptr<const uint8_t>(v, v->data());
  return Status::Ok();
}

Status GpuHasher::SumBatch(const uint8_t* base, const uint64_t* off, const uint64_t* len,
                           size_t n, Ref* refs) {
  if (n == 0) return Status::Ok();
  std::lock_guard<std::mutex> g(mu_);
  if (!h_ && !(h_ = hasher_acquire(device_))) return Status::Err(BSG_EDEVICE, "bsg_hasher_new");
  static const uint8_t empty = 0;
  static_assert(sizeof(Ref) == 32, "Ref is 32 packed bytes");
  int rc = bsg_hasher_sum(h_, base ? base : &empty, off, len, (uint32_t)n,
                          reinterpret_cast<uint8_t*>(refs));
  return rc ? Status::Err(rc, std::string("sha256: ") + bsg_errstr(rc)) : Status::Ok();
}

Status GpuHasher::SumPtrs(const uint8_t* const* ptrs, const uint64_t* len, size_t n, Ref* refs) {
  if (n == 0) return Status::Ok();
  std::lock_guard<std::mutex> g(mu_);
  if (!h_ && !(h_ = hasher_acquire(device_))) return Status::Err(BSG_EDEVICE, "bsg_hasher_new");
  int rc = bsg_hasher_sum_ptrs(h_, ptrs, len, (uint32_t)n, reinterpret_cast<uint8_t*>(refs));
  return rc ? Status::Err(rc, std::string("sha256: ") + bsg_errstr(rc)) : Status::Ok();
}

Status GpuHasher::Sum(const uint8_t* data, size_t n, Ref* out) {
  const uint64_t off = 0, len = n;
  return SumBatch(data, &off, &len, 1, out);
}

Status MemStore::Get(const Ref& ref, std::vector<uint8_t>* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = blobs_.find(ref);
  if (it == blobs_.end()) return Status::Err(kNotFound, "not found");
  out->assign(it->second.bytes(), it->second.bytes() + it->second.size);
  return Status::Ok();
}

Status MemStore::GetBlob(const Ref& ref, Blob* out) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = blobs_.find(ref);
  if (it == blobs_.end()) return Status::Err(kNotFound, "not found");
  *out = it->second;
  return Status::Ok();
}

Status MemStore::Put(const uint8_t* data, size_t n, Ref* ref, bool* added) {  // mem.go:62-76
  Ref r;
  Status s = hasher_.Sum(data, n, &r);
  if (!s.ok()) return s;
  if (ref) *ref = r;
  return PutWithRef(r, data, n, added);
}

Status MemStore::PutWithRef(const Ref& ref, const uint8_t* data, size_t n, bool* added) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = blobs_.find(ref);
  bool add = it == blobs_.end();
  if (add) {  // a caller's buffer: keep a copy
    std::shared_ptr<uint8_t> own(new uint8_t[n ? n : 1], std::default_delete<uint8_t[]>());
    if (n) std::memcpy(own.get(), data, n);
    blobs_.emplace(ref, Blob{std::move(own), n});
  }
  if (added) *added = add;
  return Status::Ok();
}

Status MemStore::PutBlob(const Ref& ref, const Blob& b, bool* added, uint64_t) {  // mem.go:62-76
  std::lock_guard<std::mutex> g(mu_);
  const bool add = blobs_.emplace(ref, b).second;
  if (add && b.base_size > b.size) {  // an alias into a larger buffer: account for its share
    Share& sh = shares_[Owner(b.data)];
    sh.base_size = b.base_size;
    sh.live += b.size;
    sh.refs.push_back(ref);
  }
  if (added) *added = add;
  return Status::Ok();
}

// Copies the blobs still aliasing a sealed buffer into buffers of their own once they keep
// less than half of it alive; the buffer is then freed with its last other reference.
void MemStore::MaybeCompact(std::map<Owner, Share, std::owner_less<Owner>>::iterator it) {
  Share& sh = it->second;
  if (!sh.sealed || sh.live * 2 >= sh.base_size) return;
  for (const Ref& r : sh.refs) {
    auto b = blobs_.find(r);
    if (b == blobs_.end()) continue;  // deleted
    std::shared_ptr<uint8_t> own(new uint8_t[b->second.size ? b->second.size : 1],
                                 std::default_delete<uint8_t[]>());
    if (b->second.size) std::memcpy(own.get(), b->second.bytes(), b->second.size);
    b->second = Blob{std::move(own), b->second.size, 0};
  }
  shares_.erase(it);
}

void MemStore::Seal(const Blob& whole) {
  std::lock_guard<std::mutex> g(mu_);
  auto it = shares_.find(Owner(whole.data));
  if (it == shares_.end()) return;
  it->second.sealed = true;
  MaybeCompact(it);
}

size_t MemStore::HeldBytes() const {
  std::lock_guard<std::mutex> g(mu_);
  size_t n = 0;
  for (const auto& kv : blobs_)
    if (kv.second.base_size <= kv.second.size) n += kv.second.size;
  for (const auto& kv : shares_) n += kv.second.base_size;
  return n;
}

Status MemStore::ListRefs(const Ref& start, const std::function<Status(const Ref&)>& f) {
  std::vector<Ref> refs;
  {
    std::lock_guard<std::mutex> g(mu_);
    for (auto it = blobs_.upper_bound(start); it != blobs_.end(); ++it) refs.push_back(it->first);
  }
  for (const Ref& r : refs) {
    Status s = f(r);
    if (!s.ok()) return s;
  }
  return Status::Ok();
}

Status MemStore::Delete(const Ref& ref) {  // mem.go:79-85
  std::lock_guard<std::mutex> g(mu_);
  auto b = blobs_.find(ref);
  if (b == blobs_.end()) return Status::Ok();
  const Blob blob = b->second;
  blobs_.erase(b);
  if (blob.base_size > blob.size) {
    auto it = shares_.find(Owner(blob.data));
    if (it != shares_.end()) {
      Share& sh = it->second;
      sh.live -= blob.size;
      sh.refs.erase(std::find(sh.refs.begin(), sh.refs.end(), ref));
      if (sh.refs.empty()) {
        shares_.erase(it);
      } else {
        MaybeCompact(it);
      }
    }
  }
  return Status::Ok();
}

size_t MemStore::Size() const {
  std::lock_guard<std::mutex> g(mu_);
  return blobs_.size();
}

namespace split {

// ---------------------------------------------------------------------------------------------
// proto3 wire format of split.Node / split.Child, as Go's proto.Marshal writes it: fields in
// number order, zero-valued scalars omitted, repeated messages length-delimited.
// ---------------------------------------------------------------------------------------------
namespace {
void put_varint(std::string& o, uint64_t v) {
  while (v >= 0x80) {
    o.push_back((char)(v | 0x80));
    v >>= 7;
  }
  o.push_back((char)v);
}
std::string child_bytes(const Child& c) {
  std::string o;
  o.push_back(0x0a);
  put_varint(o, 32);
  o.append(reinterpret_cast<const char*>(c.ref.data()), 32);
  if (c.offset) {
    o.push_back(0x10);
    put_varint(o, c.offset);
  }
  return o;
}
bool get_varint(const uint8_t*& p, const uint8_t* e, uint64_t* v) {
  uint64_t x = 0;
  for (int s = 0; s < 64 && p < e; s += 7) {
    const uint8_t b = *p++;
    x |= (uint64_t)(b & 0x7f) << s;
    if (b < 0x80) {
      *v = x;
      return true;
    }
  }
  return false;
}
bool parse_child(const uint8_t* p, const uint8_t* e, Child* c) {
  while (p < e) {
    uint64_t tag, v;
    if (!get_varint(p, e, &tag)) return false;
    if (tag == 0x0a) {
      if (!get_varint(p, e, &v) || v > (uint64_t)(e - p)) return false;
      std::memset(c->ref.data(), 0, 32);
      std::memcpy(c->ref.data(), p, std::min<uint64_t>(v, 32));  // bs.RefFromBytes
      p += v;
    } else if (tag == 0x10) {
      if (!get_varint(p, e, &c->offset)) return false;
    } else {
      return false;
    }
  }
  return true;
}
}  // namespace

std::string Node::Marshal() const {
  std::string o;
  for (const Child& c : nodes) {
    std::string b = child_bytes(c);
    o.push_back(0x0a);
    put_varint(o, b.size());
    o += b;
  }
  for (const Child& c : leaves) {
    std::string b = child_bytes(c);
    o.push_back(0x12);
    put_varint(o, b.size());
    o += b;
  }
  if (offset) {
    o.push_back(0x18);
    put_varint(o, offset);
  }
  if (size) {
    o.push_back(0x20);
    put_varint(o, size);
  }
  return o;
}

bool Node::Unmarshal(const uint8_t* p, size_t n) {
  const uint8_t* e = p + n;
  nodes.clear();
  leaves.clear();
  offset = size = 0;
  while (p < e) {
    uint64_t tag, v;
    if (!get_varint(p, e, &tag)) return false;
    if (tag == 0x0a || tag == 0x12) {
      if (!get_varint(p, e, &v) || v > (uint64_t)(e - p)) return false;
      Child c;
      if (!parse_child(p, p + v, &c)) return false;
      (tag == 0x0a ? nodes : leaves).push_back(c);
      p += v;
    } else if (tag == 0x18) {
      if (!get_varint(p, e, &offset)) return false;
    } else if (tag == 0x20) {
      if (!get_varint(p, e, &size)) return false;
    } else {
      return false;
    }
  }
  return true;
}

// ---------------------------------------------------------------------------------------------
// Writer
// ---------------------------------------------------------------------------------------------
struct Writer::Wrapped {  // split.nodeWrapper: a finished Node whose children are stored
  Node node;
};
struct Writer::TBNode {   // hashsplit.TreeBuilderNode
  std::vector<std::shared_ptr<Wrapped>> nodes;
  std::vector<Child> chunks;  // refs (the bytes are already Put) with their lengths in offset
  uint64_t size = 0, offset = 0;
};

Writer::Writer(int device) : hasher_(device) {}

// A process-wide pool of streaming contexts, keyed by (device, bits, min_size, tile): a
// split.Writer per file (fs.Dir.AddDir) would otherwise pay for three engines and their pinned
// staging on every NewWriter. A context goes back with bsg_reset when its Writer is destroyed.
namespace {
struct CtxKey {
  int device;
  uint32_t bits, min_size;
  size_t tile;
  bool operator<(const CtxKey& o) const {
    return std::tie(device, bits, min_size, tile) < std::tie(o.device, o.bits, o.min_size, o.tile);
  }
};
std::mutex g_pool_mu;
std::map<CtxKey, std::vector<bsg_ctx*>>& ctx_pool() {
  static auto* pool = new std::map<CtxKey, std::vector<bsg_ctx*>>();  // never destroyed:
  return *pool;  // pooled contexts live until exit (their HIP runtime may be torn down first)
}
constexpr size_t kPoolPerKey = 4;

bsg_ctx* ctx_acquire(const CtxKey& k, const bsg_params* p, int* rc) {
  {
    std::lock_guard<std::mutex> g(g_pool_mu);
    auto& v = ctx_pool()[k];
    if (!v.empty()) {
      bsg_ctx* c = v.back();
      v.pop_back();
      *rc = BSG_OK;
      return c;
    }
  }
  bsg_ctx* c = bsg_open(k.device, p, nullptr, rc);
  if (c && k.tile && (*rc = bsg_set_tile(c, k.tile)) != BSG_OK) {
    bsg_free(c);
    return nullptr;
  }
  return c;
}

void ctx_release(const CtxKey& k, bsg_ctx* c) {
  if (!c) return;
  if (bsg_reset(c) == BSG_OK) {
    std::lock_guard<std::mutex> g(g_pool_mu);
    auto& v = ctx_pool()[k];
    if (v.size() < kPoolPerKey) {
      v.push_back(c);
      return;
    }
  }
  bsg_free(c);
}
}  // namespace

std::unique_ptr<Writer> Writer::New(Store* st, const Options& opt, Status* err) {
  Status dummy;
  if (!err) err = &dummy;
  if (!st) {
    *err = Status::Err(BSG_EINVAL, "nil store");
    return nullptr;
  }
  std::unique_ptr<Writer> w(new Writer(opt.device));
  w->st_ = st;
  w->rp_ = dynamic_cast<RefPutter*>(st);
  if (w->rp_) w->group_ = w->rp_->OpenGroup();
  w->opt_ = opt;
  if (w->opt_.fanout == 0) w->opt_.fanout = 1;
  bsg_params p;
  p.split_bits = opt.bits;
  p.min_size = (uint32_t)std::max(opt.min_size, 0);
  p.fanout = w->opt_.fanout;
  p.reserved = 0;
  int rc = 0;
  w->ctx_ = ctx_acquire(CtxKey{opt.device, p.split_bits, p.min_size, opt.tile}, &p, &rc);
  if (!w->ctx_) {
    *err = Status::Err(rc, std::string("bsg_open: ") + bsg_errstr(rc));
    return nullptr;
  }
  *err = Status::Ok();
  return w;
}

namespace {
double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
}  // namespace

struct Writer::Bg {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::vector<bsg_chunk> job;
  bool pending = false, stop = false;
  Status st;  // the first error not yet returned by Join
};

Writer::~Writer() {
  if (bg_) {
    {
      std::lock_guard<std::mutex> g(bg_->mu);
      bg_->stop = true;
      bg_->cv.notify_all();
    }
    bg_->th.join();  // after its last job
  }
  static const bool debug = std::getenv("BSG_DEBUG_WRITER") != nullptr;
  if (debug)
    std::fprintf(stderr,
                 "bsgpu writer: copy %.1f ms, drain %.1f ms (waited %.1f), node hashes %.1f ms in "
                 "%llu calls, close %.1f ms\n",
                 tm_.copy * 1e3, tm_.drain * 1e3, tm_.join * 1e3, tm_.hash * 1e3,
                 (unsigned long long)tm_.hash_calls, tm_.close * 1e3);
  if (rp_) rp_->CloseGroup(group_);
  if (ctx_)
    ctx_release(CtxKey{opt_.device, opt_.bits, (uint32_t)std::max(opt_.min_size, 0), opt_.tile},
                ctx_);
}

Status Writer::PutProto(const Node& node, Ref* ref) {
  const std::string b = node.Marshal();
  bool added;
  if (rp_) {
    Status s = hasher_.Sum(reinterpret_cast<const uint8_t*>(b.data()), b.size(), ref);
    if (!s.ok()) return s;
    return rp_->PutWithRef(*ref, reinterpret_cast<const uint8_t*>(b.data()), b.size(), &added);
  }
  return st_->Put(reinterpret_cast<const uint8_t*>(b.data()), b.size(), ref, &added);
}

Status Writer::PutProtos(const std::vector<const Node*>& nodes, std::vector<Ref>* refs) {
  refs->assign(nodes.size(), Ref{});
  if (nodes.empty()) return Status::Ok();
  // A node is stored only once everything under it is (split/split.go:71-77 Puts a node's
  // chunks before PutProto of the node): wait for this Writer's write-behind blobs first.
  if (rp_) {
    Status f = rp_->Flush(group_);
    if (!f.ok()) return f;
  }
  if (!rp_) {  // the store hashes each blob itself
    for (size_t i = 0; i < nodes.size(); ++i) {
      Status s = PutProto(*nodes[i], &(*refs)[i]);
      if (!s.ok()) return s;
    }
    return Status::Ok();
  }
  std::string packed;
  std::vector<uint64_t> off(nodes.size()), len(nodes.size());
  for (size_t i = 0; i < nodes.size(); ++i) {
    const std::string b = nodes[i]->Marshal();
    off[i] = packed.size();
    len[i] = b.size();
    packed += b;
  }
  const double t0 = now_s();
  Status s = hasher_.SumBatch(reinterpret_cast<const uint8_t*>(packed.data()), off.data(),
                              len.data(), nodes.size(), refs->data());
  tm_.hash += now_s() - t0;
  tm_.hash_calls++;
  if (!s.ok()) return s;
  for (size_t i = 0; i < nodes.size(); ++i) {
    bool added;
    s = rp_->PutWithRef((*refs)[i], reinterpret_cast<const uint8_t*>(packed.data()) + off[i],
                        len[i], &added);
    if (!s.ok()) return s;
  }
  return Status::Ok();
}

Status Writer::F(TBNode& n, std::shared_ptr<Wrapped>* out) {  // split/split.go:52-81
  auto w = std::make_shared<Wrapped>();
  uint64_t offset = n.offset;
  w->node.offset = n.offset;
  w->node.size = n.size;
  std::vector<const Node*> kids;
  for (const auto& child : n.nodes) kids.push_back(&child->node);
  std::vector<Ref> refs;
  Status s = PutProtos(kids, &refs);  // split.go:61-69, all children in one GPU call
  if (!s.ok()) return s;
  for (size_t i = 0; i < n.nodes.size(); ++i) {
    w->node.nodes.push_back(Child{refs[i], offset});
    offset += n.nodes[i]->node.size;
  }
  for (const Child& c : n.chunks) {  // chunks were Put on arrival; c.offset holds the length
    w->node.leaves.push_back(Child{c.ref, offset});
    offset += c.offset;
  }
  *out = std::move(w);
  return Status::Ok();
}

Status Writer::Add(const Ref& ref, uint64_t len, unsigned level) {  // TreeBuilder.Add
  if (levels_.empty()) levels_.emplace_back(new TBNode());
  levels_[0]->chunks.push_back(Child{ref, len});
  for (auto& n : levels_) n->size += len;
  for (unsigned i = 0; i < level; ++i) {
    if (i == levels_.size() - 1) {
      auto* top = new TBNode();
      top->size = levels_[i]->size;
      top->offset = levels_[i]->offset;
      levels_.emplace_back(top);
    }
    std::shared_ptr<Wrapped> w;
    Status s = F(*levels_[i], &w);
    if (!s.ok()) return s;
    levels_[i + 1]->nodes.push_back(std::move(w));
    auto* fresh = new TBNode();
    fresh->offset = levels_[i + 1]->offset + levels_[i + 1]->size;
    levels_[i].reset(fresh);
  }
  return Status::Ok();
}

Status Writer::SetStreamBase(uint64_t base) {
  if (end_ != base_ || closed_) return Status::Err(BSG_ESTATE, "stream base after the first Write");
  const int rc = bsg_set_stream_base(ctx_, base);
  if (rc) return Status::Err(rc, std::string("bsg_set_stream_base: ") + bsg_errstr(rc));
  base_ = end_ = emitted_ = base;
  return Status::Ok();
}

size_t Writer::TakeRecords(std::vector<bsg_chunk>* out) {
  out->clear();
  const size_t n = bsg_pending(ctx_);
  if (!n) return 0;
  out->resize(n);
  out->resize(bsg_drain(ctx_, out->data(), n));
  return out->size();
}

Status Writer::Drain() {
  TakeRecords(&drained_);
  return Process(drained_);
}

void Writer::Submit(std::vector<bsg_chunk>* recs) {
  if (!bg_) {
    bg_.reset(new Bg());
    bg_->th = std::thread([this] {
      Bg& b = *bg_;
      std::unique_lock<std::mutex> g(b.mu);
      for (;;) {
        b.cv.wait(g, [&] { return b.pending || b.stop; });
        if (!b.pending) return;  // stopping
        g.unlock();
        const double t0 = now_s();
        Status s = Process(b.job);
        tm_.drain += now_s() - t0;
        g.lock();
        if (!s.ok() && b.st.ok()) b.st = s;
        b.pending = false;
        b.cv.notify_all();
      }
    });
  }
  std::lock_guard<std::mutex> g(bg_->mu);
  bg_->job.swap(*recs);
  bg_->pending = true;
  bg_->cv.notify_all();
}

Status Writer::Join() {
  if (!bg_) return Status::Ok();
  std::unique_lock<std::mutex> g(bg_->mu);
  bg_->cv.wait(g, [&] { return !bg_->pending; });
  Status s = bg_->st;
  bg_->st = Status::Ok();
  return s;
}

Status Writer::Process(const std::vector<bsg_chunk>& recs) {
  const size_t got = recs.size();
  for (size_t i = 0; i < got; ++i) {
    const bsg_chunk& c = recs[i];
    if (c.offset != emitted_ || c.offset + c.len > end_)
      return Status::Err(BSG_EDEVICE, "chunk records out of order");
    // the chunk's bytes: an alias of the piece that holds them, or (a chunk across pieces)
    // gathered into a buffer of its own
    Blob blob;
    blob.size = c.len;
    uint64_t skip = c.offset - base_;
    size_t k = 0;
    while (skip >= pieces_[k].size) skip -= pieces_[k++].size;
    if (skip + c.len <= pieces_[k].size) {
      blob.data = std::shared_ptr<const uint8_t>(pieces_[k].buf, pieces_[k].buf.get() + skip);
      blob.base_size = pieces_[k].size;
    } else {
      std::shared_ptr<uint8_t> own(new uint8_t[c.len], std::default_delete<uint8_t[]>());
      uint64_t done = 0;
      for (; done < c.len; ++k, skip = 0) {
        const uint64_t take = std::min<uint64_t>(c.len - done, pieces_[k].size - skip);
        std::memcpy(own.get() + done, pieces_[k].buf.get() + skip, take);
        done += take;
      }
      blob.data = std::move(own);
    }
    Ref ref;
    std::memcpy(ref.data(), c.ref, 32);
    bool added;
    Status s = rp_ ? rp_->PutBlob(ref, blob, &added, group_)        // GPU ref, no re-hash
                   : st_->Put(blob.bytes(), c.len, &ref, &added);  // store computes the ref
    if (!s.ok()) return s;
    emitted_ += c.len;
    while (!pieces_.empty() && base_ + pieces_.front().size <= emitted_) {  // fully emitted
      base_ += pieces_.front().size;
      if (rp_) rp_->Seal(Blob{pieces_.front().buf, pieces_.front().size, 0});
      pieces_.pop_front();
    }
    s = Add(ref, c.len, c.level / opt_.fanout);  // split/split.go:86
    if (!s.ok()) return s;
  }
  return Status::Ok();
}

// A piece buffer. Large ones are their own anonymous mapping with transparent huge pages
// requested: they are written once, kept by the store, and a fresh 4 KiB-page heap buffer
// costs a page fault per 4 KiB on its first write (the largest cost of a Write before).
// Released mappings are kept for the next Writer in a process-wide pool of at most
// kPiecePoolMax bytes (a server whose stores release their blobs — store/file after write-behind,
// a dropped store/mem — reuses them): a fresh mapping costs its page faults plus the kernel
// zeroing every page before the Write's copy writes it again, a second pass over host memory
// (round 6: the Writer's copies took 25-30 ms per GiB against 7-10 for the raw path's,
// profiles/r06_c1_copy_ab.log).
namespace {
constexpr size_t kPieceHuge = 2ull << 20;
constexpr size_t kPiecePoolMax = 1ull << 30;
struct PiecePool {
  std::mutex mu;
  std::multimap<size_t, void*> free;  // mapping length -> mapping
  size_t bytes = 0;
};
PiecePool& piece_pool() {
  static auto* p = new PiecePool();  // never destroyed: mappings live until exit
  return *p;
}
void piece_release(void* m, size_t len) {
  PiecePool& pp = piece_pool();
  {
    std::lock_guard<std::mutex> g(pp.mu);
    if (pp.bytes + len <= kPiecePoolMax) {
      pp.free.emplace(len, m);
      pp.bytes += len;
      return;
    }
  }
  ::munmap(m, len);
}
void* piece_take(size_t len) {
  PiecePool& pp = piece_pool();
  std::lock_guard<std::mutex> g(pp.mu);
  auto it = pp.free.find(len);
  if (it == pp.free.end()) return nullptr;
  void* m = it->second;
  pp.free.erase(it);
  pp.bytes -= len;
  return m;
}
}  // namespace

static std::shared_ptr<uint8_t> alloc_piece(size_t n) {
  if (n >= kPieceHuge) {
    const size_t len = (n + kPieceHuge - 1) & ~(kPieceHuge - 1);
    void* m = piece_take(len);
    if (!m) {
      m = ::mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS, -1, 0);
      if (m == MAP_FAILED) m = nullptr;
      if (m) (void)::madvise(m, len, MADV_HUGEPAGE);
    }
    if (m)
      return std::shared_ptr<uint8_t>(static_cast<uint8_t*>(m),
                                      [len](uint8_t* q) { piece_release(q, len); });
  }
  return std::shared_ptr<uint8_t>(new (std::nothrow) uint8_t[n ? n : 1],
                                  std::default_delete<uint8_t[]>());
}

// Copies p[0..n) into dst (the Writer's piece) and, through the zero-copy window, into the
// context's pinned staging: one read of the caller's bytes feeds both copies, streamed into the
// two destinations with non-temporal stores (bsg::copy_nt2; with BSG_KNOB_COPY_NT off, each
// thread copies a 64 KiB slice into the piece, then from there, still in cache, into the
// window), on the process-wide copy pool (host_pool.h: BSG_COPY_THREADS threads shared by all
// Writers).
Status Writer::Copy(const uint8_t* p, size_t n, uint8_t* dst) {
  size_t done = 0;
  while (done < n) {
    uint8_t* win = nullptr;
    size_t cap = 0;
    int rc = bsg_write_window(ctx_, &win, &cap);
    if (rc) return Status::Err(rc, std::string("bsg_write_window: ") + bsg_errstr(rc));
    const size_t k = std::min(cap, n - done);
    const uint8_t* src = p + done;
    uint8_t* d1 = dst + done;
    const bool use_nt = bsg::copy_nt_enabled();
    auto work = [=](size_t lo, size_t hi) {
      if (use_nt) {  // one read of the caller's bytes, streamed into the piece and the stage
        bsg::copy_nt2(d1 + lo, win + lo, src + lo, hi - lo);
        return;
      }
      constexpr size_t kSlice = 64 << 10;
      for (size_t o = lo; o < hi; o += kSlice) {
        const size_t m = std::min(kSlice, hi - o);
        std::memcpy(d1 + o, src + o, m);
        std::memcpy(win + o, d1 + o, m);
      }
    };
    constexpr size_t kPerThread = 2ull << 20;
    const size_t nt = std::min<size_t>((size_t)bsg::copy_threads(), k / kPerThread);
    if (nt <= 1) {
      work(0, k);
    } else {  // kCopySlice slices taken dynamically (a late or slow thread takes fewer)
      constexpr size_t sl = bsg::kCopySlice;
      bsg::parallel_for((k + sl - 1) / sl,
                        [&](size_t t) { work(t * sl, std::min(k, t * sl + sl)); });
    }
    rc = bsg_write_commit(ctx_, k);
    if (rc) return Status::Err(rc, std::string("bsg_write_commit: ") + bsg_errstr(rc));
    done += k;
  }
  return Status::Ok();
}

Status Writer::Write(const uint8_t* p, size_t n, size_t* written) {
  if (written) *written = 0;
  if (closed_) return Status::Err(BSG_ESTATE, "write after close");
  if (!sticky_.ok()) return sticky_;
  // the previous Write's records are processed; this Write's ready records go to the background
  // thread, which reads only pieces of earlier Writes while this one is copied into a new piece
  const double t1 = now_s();
  Status s = Join();
  tm_.join += now_s() - t1;
  if (!s.ok()) return sticky_ = s;
  std::vector<bsg_chunk> recs;
  TakeRecords(&recs);
  uint8_t* dst = nullptr;
  if (n) {
    Piece piece{alloc_piece(n), n};
    if (!piece.buf) return sticky_ = Status::Err(BSG_ENOMEM, "piece allocation");
    dst = piece.buf.get();
    pieces_.push_back(std::move(piece));
    end_ += n;
  }
  if (!recs.empty()) Submit(&recs);
  if (n) {
    const double t0 = now_s();
    // (Registering the piece and writing it with bsg_write_pinned, to skip the staging copy,
    // measured slower: 12-13 GiB/s against 15-25 on 4 GiB in 32 MiB Writes)
    s = Copy(p, n, dst);
    tm_.copy += now_s() - t0;
    if (!s.ok()) {
      Join();  // the background thread must not outlive the error path's state changes
      return sticky_ = s;
    }
  }
  if (written) *written = n;
  return Status::Ok();
}

Status Writer::Close() {  // split/split.go:104-126
  if (closed_) return sticky_;
  closed_ = true;
  if (!sticky_.ok()) return sticky_;
  const double t0 = now_s();
  struct Clock {  // close time, however Close returns
    double t0;
    double* acc;
    ~Clock() { *acc += now_s() - t0; }
  } clock{t0, &tm_.close};
  Status js = Join();
  if (!js.ok()) return sticky_ = js;
  // the last tiles finish one by one: each one's chunks are Put (background thread) while the
  // next is still on the device
  double td = now_s();
  int rc = bsg_close_begin(ctx_);
  for (size_t left = 1; rc == BSG_OK && left;) {
    rc = bsg_close_step(ctx_, &left);
    tm_.close_dev += now_s() - td;
    if (rc) break;
    const double tj = now_s();
    Status s = Join();
    td = now_s();
    tm_.join += td - tj;
    if (!s.ok()) return sticky_ = s;
    std::vector<bsg_chunk> recs;
    if (TakeRecords(&recs)) Submit(&recs);
  }
  if (rc) {
    Join();
    return sticky_ = Status::Err(rc, std::string("bsg_close: ") + bsg_errstr(rc));
  }
  Status s = Join();
  if (!s.ok()) return sticky_ = s;
  s = Drain();
  if (!s.ok()) return sticky_ = s;
  if (levels_.empty()) return Status::Ok();  // no input: Root stays bs.Zero
  // TreeBuilder.Root(): fold every non-empty level below the top into its parent
  for (size_t i = 0; i + 1 < levels_.size(); ++i) {
    TBNode& n = *levels_[i];
    if (n.chunks.empty() && n.nodes.empty()) continue;
    std::shared_ptr<Wrapped> w;
    if (!(s = F(n, &w)).ok()) return sticky_ = s;
    levels_[i + 1]->nodes.push_back(std::move(w));
  }
  std::shared_ptr<Wrapped> root;
  if (levels_.size() == 1) {
    if (!(s = F(*levels_[0], &root)).ok()) return sticky_ = s;
  } else {
    TBNode& top = *levels_.back();
    if (top.nodes.size() > 1) {
      if (!(s = F(top, &root)).ok()) return sticky_ = s;
    } else {
      root = top.nodes[0];  // prune would-be roots with a single child
      while (root->node.nodes.size() == 1) {
        std::vector<uint8_t> b;
        if (!(s = st_->Get(root->node.nodes[0].ref, &b)).ok()) return sticky_ = s;
        auto next = std::make_shared<Wrapped>();
        if (!next->node.Unmarshal(b.data(), b.size()))
          return sticky_ = Status::Err(BSG_EINVAL, "bad tree node");
        root = next;
      }
    }
  }
  // the root last, once every blob and node under it is stored (write-behind stores)
  if (rp_ && !(s = rp_->Flush(group_)).ok()) return sticky_ = s;
  s = PutProto(root->node, &root_);
  if (!s.ok()) return sticky_ = s;
  levels_.clear();
  return Status::Ok();
}

// ---------------------------------------------------------------------------------------------
// Reader (split/split.go:173-303)
// ---------------------------------------------------------------------------------------------
namespace {
Status get_node(Store* g, const Ref& ref, Node* n) {
  std::vector<uint8_t> b;
  Status s = g->Get(ref, &b);
  if (!s.ok()) return s;
  if (!n->Unmarshal(b.data(), b.size())) return Status::Err(BSG_EINVAL, "bad tree node");
  return Status::Ok();
}
}  // namespace

Status Protect(Store* g, const Ref& ref, std::vector<ProtectPair>* out) {  // split.go:306-322
  out->clear();
  Node n;
  Status s = get_node(g, ref, &n);
  if (!s.ok()) return s;
  for (const Child& c : n.nodes) out->push_back(ProtectPair{c.ref, true});
  for (const Child& c : n.leaves) out->push_back(ProtectPair{c.ref, false});
  return Status::Ok();
}

std::unique_ptr<Reader> Reader::New(Store* g, const Ref& root, Status* err, bool verify,
                                    int device) {
  Status dummy;
  if (!err) err = &dummy;
  Node n;
  Status s = get_node(g, root, &n);
  if (!s.ok()) {
    *err = Status::Err(s.code, "getting root ref " + RefString(root) + ": " + s.msg);
    return nullptr;
  }
  std::unique_ptr<Reader> r(new Reader());
  r->g_ = g;
  r->verify_ = verify;
  r->device_ = device;
  if (const int64_t wb = bsg_debug_get(BSG_KNOB_VERIFY_WINDOW))  // tests: small windows
    r->window_bytes_ = (uint64_t)wb;
  r->stack_.push_back(std::move(n));
  *err = Status::Ok();
  return r;
}

Reader::~Reader() {
  if (ahead_.valid()) ahead_.wait();  // the background window uses this Reader's store, hasher
  static const bool debug = std::getenv("BSG_DEBUG_READER") != nullptr;
  if (debug && verify_)
    std::fprintf(stderr,
                 "bsgpu reader: %llu windows on the reading thread (%.1f ms), %llu ahead; "
                 "%.1f MiB verified: walk %.1f ms, fetch %.1f ms, hash %.1f ms; reads waited "
                 "%.1f ms for windows ahead\n",
                 (unsigned long long)tm_.sync_windows, tm_.sync * 1e3,
                 (unsigned long long)tm_.ahead_windows, tm_.bytes / 1048576.0, tm_.walk * 1e3,
                 tm_.fetch * 1e3, tm_.hash * 1e3, tm_.wait * 1e3);
}

// Verify mode. The next leaf node of the walk `cur` (a node with leaves), fetching the internal
// nodes on the way; *done at the end of the tree.
Status Reader::NextLeafNode(std::vector<Frame>* cur, Node* out, bool* done) {
  *done = false;
  while (!cur->empty()) {
    Frame& f = cur->back();
    if (f.next >= f.node.nodes.size()) {
      cur->pop_back();
      continue;
    }
    const Ref ref = f.node.nodes[f.next++].ref;
    Node n;
    Status s = get_node(g_, ref, &n);
    if (!s.ok()) return Status::Err(s.code, "getting tree node: " + s.msg);
    if (!n.leaves.empty()) {
      *out = std::move(n);
      return Status::Ok();
    }
    cur->push_back(Frame{std::move(n), 0});
  }
  *done = true;
  return Status::Ok();
}

// Verify mode: `first` (if given) and the leaf nodes after it in the walk, up to `budget` bytes:
// their chunks fetched through Store::GetBlob (store/mem hands out its own Blobs, no copy) and
// checked in one batched GPU SHA-256 call (bsg_hasher_sum_ptrs: bsg_engine_hash mode, the
// long chunks on wave-mode chains). Runs on the reading thread or on the background one.
Reader::Window Reader::VerifyRun(std::vector<Frame> cur, const Node* first, uint64_t budget) {
  Window w;
  double t = now_s();
  auto lap = [&t](double* acc) {
    const double t1 = now_s();
    *acc += t1 - t;
    t = t1;
  };
  std::vector<Node> nodes;
  uint64_t total = 0;
  if (first) {
    nodes.push_back(*first);
    total = first->size;
  }
  while (total < budget) {
    Node n;
    bool done = false;
    w.st = NextLeafNode(&cur, &n, &done);
    if (!w.st.ok()) return w;
    if (done) {
      w.end = true;
      break;
    }
    total += n.size;
    nodes.push_back(std::move(n));
  }
  w.cursor = std::move(cur);
  w.bytes = total;
  lap(&w.t_walk);
  for (const Node& n : nodes) w.covered.push_back(n.offset);
  std::vector<std::vector<Blob>> chunks(nodes.size());
  std::vector<std::pair<size_t, size_t>> all;  // (leaf node, leaf)
  for (size_t i = 0; i < nodes.size(); ++i) {
    chunks[i].resize(nodes[i].leaves.size());
    for (size_t k = 0; k < nodes[i].leaves.size(); ++k) all.emplace_back(i, k);
  }
  // fetched on up to 8 threads (store/file reads a file per chunk; store/mem only looks up)
  std::vector<Status> errs(std::min<size_t>(8, std::max<size_t>(1, all.size() / 64)));
  auto fetch = [&](size_t t) {
    for (size_t x = t; x < all.size(); x += errs.size()) {
      const size_t i = all[x].first, k = all[x].second;
      Status s = g_->GetBlob(nodes[i].leaves[k].ref, &chunks[i][k]);
      if (!s.ok()) {
        errs[t] = Status::Err(s.code, "getting chunk: " + s.msg);
        return;
      }
    }
  };
  bsg::parallel_for(errs.size(), fetch);
  lap(&w.t_fetch);
  for (const Status& e : errs)
    if (!e.ok()) {
      w.st = e;
      return w;
    }
  std::vector<const uint8_t*> ptrs;
  std::vector<uint64_t> lens;
  std::vector<const Ref*> want;
  for (size_t i = 0; i < nodes.size(); ++i)
    for (size_t k = 0; k < nodes[i].leaves.size(); ++k) {
      ptrs.push_back(chunks[i][k].bytes());
      lens.push_back(chunks[i][k].size);
      want.push_back(&nodes[i].leaves[k].ref);
    }
  std::vector<Ref> refs(ptrs.size());
  Status s = hasher_->SumPtrs(ptrs.data(), lens.data(), ptrs.size(), refs.data());
  lap(&w.t_hash);
  if (!s.ok()) {
    w.st = Status::Err(s.code, "verifying chunks: " + s.msg);
    return w;
  }
  for (size_t k = 0; k < refs.size(); ++k)
    if (refs[k] != *want[k]) {
      w.st = Status::Err(kCorrupt, "chunk " + RefString(*want[k]) + " fails verification");
      return w;
    }
  for (size_t i = 0; i < nodes.size(); ++i) w.leaves[nodes[i].offset] = std::move(chunks[i]);
  return w;
}

// Verify mode: cache_ = the verified chunks of stack_.back(). From the current window if it
// holds them; else from the window verified in the background, if it does; else a window is
// verified here, starting at this leaf node (the first read, or after a seek). Each time a
// window is taken, the one after it is started in the background.
Status Reader::TakeLeaf() {
  const uint64_t at = stack_.back().offset;
  // Sequential reading (the first leaf node, or the one right after the last taken) verifies
  // whole windows and reads ahead; a read elsewhere (a seek) verifies just its leaf node, so a
  // random or backward read costs one leaf node's fetch and hash, not a 256 MiB window.
  const bool sequential = at == next_leaf_;
  next_leaf_ = at + stack_.back().size;
  // A window in flight when the reader seeks was started for the old position: it is never
  // taken (taking it would start yet another full window from the old cursor), only waited for
  // and dropped when the next window ahead is started.
  if (!sequential && ahead_.valid()) ahead_stale_ = true;
  auto take = [&](Window&& w, bool ahead) -> Status {
    tm_.walk += w.t_walk;
    tm_.fetch += w.t_fetch;
    tm_.hash += w.t_hash;
    tm_.bytes += w.bytes;
    if (!w.st.ok()) {
      window_.clear();
      if (std::find(w.covered.begin(), w.covered.end(), at) != w.covered.end()) return w.st;
      return Status::Ok();  // a failure further on, in a window this read does not need
    }
    window_ = std::move(w.leaves);
    if (!w.end && ahead) {
      if (ahead_.valid()) {  // a stale window (see above): dropped here
        ahead_.wait();
        tm_.dropped++;
      }
      ahead_stale_ = false;
      ahead_ = std::async(std::launch::async,
                          [this, cur = std::move(w.cursor)]() mutable {
                            return VerifyRun(std::move(cur), nullptr, window_bytes_);
                          });
    }
    return Status::Ok();
  };
  auto it = window_.find(at);
  if (it == window_.end() && sequential && ahead_.valid() && !ahead_stale_) {
    const double t0 = now_s();
    Window w = ahead_.get();
    tm_.wait += now_s() - t0;
    tm_.ahead_windows++;
    Status s = take(std::move(w), true);
    if (!s.ok()) return s;
    it = window_.find(at);
  }
  if (it == window_.end()) {
    if (sequential) {  // a window read ahead for elsewhere in the stream: dropped
      if (ahead_.valid()) {
        ahead_.wait();
        tm_.dropped++;
      }
      ahead_ = std::future<Window>();
      ahead_stale_ = false;
    }
    if (!hasher_) hasher_.reset(new GpuHasher(device_));
    // the walk, positioned after stack_.back(): each internal node on the path and its child
    // after the one on the path
    std::vector<Frame> cur;
    for (size_t lvl = 0; lvl + 1 < stack_.size(); ++lvl) {
      const Node& parent = stack_[lvl];
      const uint64_t on_path = stack_[lvl + 1].offset;
      size_t c = 0;
      while (c < parent.nodes.size() && parent.nodes[c].offset <= on_path) ++c;
      cur.push_back(Frame{parent, c});
    }
    const double t0 = now_s();
    Window w = VerifyRun(std::move(cur), &stack_.back(), sequential ? window_bytes_ : 0);
    tm_.sync += now_s() - t0;
    tm_.sync_windows++;
    if (!w.st.ok()) return w.st;
    Status s = take(std::move(w), sequential);
    if (!s.ok()) return s;
    it = window_.find(at);
    if (it == window_.end()) return Status::Err(kCorrupt, "tree node offsets repeat");
  }
  cache_ = std::move(it->second);
  window_.erase(it);
  cache_valid_ = true;
  return Status::Ok();
}

Status Reader::Read(uint8_t* buf, size_t len, size_t* got, bool* eof) {
  *got = 0;
  *eof = false;
  while (len > 0) {
    for (;;) {  // unwind to a node containing pos
      const Node& node = stack_.back();
      if (pos_ >= node.offset && pos_ < node.offset + node.size) break;
      if (stack_.size() == 1) {
        *eof = true;
        return Status::Ok();
      }
      stack_.pop_back();
      cache_valid_ = false;
    }
    for (;;) {  // descend to the leaf node
      const Node& node = stack_.back();
      if (!node.leaves.empty()) break;
      if (node.nodes.empty()) return Status::Err(kCorrupt, "tree node with no children");
      size_t index = 0;
      if (pos_ > node.offset) {
        index = std::upper_bound(node.nodes.begin(), node.nodes.end(), pos_,
                                 [](uint64_t p, const Child& c) { return c.offset > p; }) -
                node.nodes.begin();
        // sort.Search (split.go:222-225) would index out of range here; a Go panic, a
        // corrupt-tree error for us
        if (index == 0) return Status::Err(kCorrupt, "tree node offsets past the read position");
        index--;
      }
      Node child;
      Status s = get_node(g_, node.nodes[index].ref, &child);
      if (!s.ok()) return Status::Err(s.code, "getting tree node: " + s.msg);
      stack_.push_back(std::move(child));
      cache_valid_ = false;
    }
    if (verify_ && !cache_valid_) {
      Status s = TakeLeaf();
      if (!s.ok()) return s;
      if (cache_.size() != stack_.back().leaves.size())
        return Status::Err(kCorrupt, "tree node offsets repeat");
    }
    const std::vector<Child>& leaves = stack_.back().leaves;
    size_t k = 0;
    while (leaves.size() - k > 1 && leaves[k + 1].offset <= pos_) ++k;
    for (; k < leaves.size() && len > 0; ++k) {
      std::vector<uint8_t> fetched;
      if (!verify_) {
        Status s = g_->Get(leaves[k].ref, &fetched);
        if (!s.ok()) return Status::Err(s.code, "getting chunk: " + s.msg);
      }
      const uint8_t* cdata = verify_ ? cache_[k].bytes() : fetched.data();
      const size_t csize = verify_ ? cache_[k].size : fetched.size();
      // offsets come from store contents: check them before indexing (Go's bounds checks
      // would panic on the same trees)
      if (leaves[k].offset > pos_ || pos_ - leaves[k].offset > csize)
        return Status::Err(kCorrupt, "leaf offsets do not match chunk sizes");
      const uint64_t skip = pos_ - leaves[k].offset;
      const size_t avail = csize - (size_t)skip;
      if (avail == 0) return Status::Err(kCorrupt, "leaf offsets do not match chunk sizes");
      const size_t take = std::min(avail, len);
      std::memcpy(buf, cdata + skip, take);
      buf += take;
      len -= take;
      *got += take;
      pos_ += take;
      if (take < avail) return Status::Ok();
    }
  }
  return Status::Ok();
}

uint64_t Reader::Seek(int64_t offset, int whence) {
  switch (whence) {
    case 0: pos_ = (uint64_t)offset; break;
    case 1: pos_ = (uint64_t)((int64_t)pos_ + offset); break;
    case 2: pos_ = (uint64_t)((int64_t)stack_.front().size + offset); break;
    default: break;
  }
  return pos_;
}

}  // namespace split
}  // namespace bs

// ---------------------------------------------------------------------------------------------
// C ABI wrappers (bsgpu.h) so the Python tests can drive the C++ host mirror.
// ---------------------------------------------------------------------------------------------
struct bsg_store {
  std::unique_ptr<bs::Store> st;
  bs::MemStore* mem = nullptr;  // set for store/mem (O(1) count)
};
struct bsg_writer {
  std::unique_ptr<bs::split::Writer> w;
};
struct bsg_reader {
  std::unique_ptr<bs::split::Reader> r;
};

extern "C" {

bsg_store* bsg_memstore_new(int device) {
  bsg_store* s = new (std::nothrow) bsg_store();
  if (!s) return nullptr;
  s->mem = new (std::nothrow) bs::MemStore(device);
  s->st.reset(s->mem);
  if (!s->mem) {
    delete s;
    return nullptr;
  }
  return s;
}
bsg_store* bsg_filestore_new(const char* root, int device) {
  if (!root || !*root) return nullptr;
  bsg_store* s = new (std::nothrow) bsg_store();
  if (!s) return nullptr;
  s->st.reset(new (std::nothrow) bs::FileStore(root, device));
  if (!s->st) {
    delete s;
    return nullptr;
  }
  return s;
}
void bsg_store_free(bsg_store* s) { delete s; }
size_t bsg_store_count(const bsg_store* s) {
  if (!s) return 0;
  if (s->mem) return s->mem->Size();
  size_t k = 0;
  s->st->ListRefs(bs::Zero, [&](const bs::Ref&) { ++k; return bs::Status::Ok(); });
  return k;
}

int bsg_filestore_set_write_behind(bsg_store* s, uint64_t bytes) {
  auto* fs = s ? dynamic_cast<bs::FileStore*>(s->st.get()) : nullptr;
  if (!fs || !bytes) return BSG_EINVAL;
  fs->SetWriteBehindLimit(bytes);
  return BSG_OK;
}

size_t bsg_store_held_bytes(const bsg_store* s) { return s && s->mem ? s->mem->HeldBytes() : 0; }

int bsg_store_get(bsg_store* s, const uint8_t ref[32], uint8_t* out, size_t cap, size_t* n) {
  if (!s || !ref || !n) return BSG_EINVAL;
  bs::Ref r;
  std::memcpy(r.data(), ref, 32);
  std::vector<uint8_t> b;
  bs::Status st = s->st->Get(r, &b);
  if (!st.ok()) return st.code;
  *n = b.size();
  if (out) std::memcpy(out, b.data(), std::min(cap, b.size()));
  return BSG_OK;
}

int bsg_store_put(bsg_store* s, const uint8_t* data, size_t n, uint8_t ref_out[32], int* added) {
  if (!s || (!data && n)) return BSG_EINVAL;
  bs::Ref r;
  bool a = false;
  bs::Status st = s->st->Put(data, n, &r, &a);
  if (!st.ok()) return st.code;
  if (ref_out) std::memcpy(ref_out, r.data(), 32);
  if (added) *added = a ? 1 : 0;
  return BSG_OK;
}

int bsg_store_put_ref(bsg_store* s, const uint8_t ref[32], const uint8_t* data, size_t n,
                      int* added) {
  if (!s || !ref || (!data && n)) return BSG_EINVAL;
  auto* rp = dynamic_cast<bs::RefPutter*>(s->st.get());
  if (!rp) return BSG_EINVAL;
  bs::Ref r;
  std::memcpy(r.data(), ref, 32);
  bool a = false;
  static const uint8_t empty = 0;
  bs::Status st = rp->PutWithRef(r, n ? data : &empty, n, &a);
  if (!st.ok()) return st.code;
  if (added) *added = a ? 1 : 0;
  return BSG_OK;
}

int bsg_store_delete(bsg_store* s, const uint8_t ref[32]) {
  if (!s || !ref) return BSG_EINVAL;
  if (!s->mem) return BSG_EINVAL;  // store/file is not a bs.DeleterStore
  bs::Ref r;
  std::memcpy(r.data(), ref, 32);
  return s->mem->Delete(r).code;
}

int bsg_split_protect(bsg_store* s, const uint8_t ref[32], uint8_t* refs, uint8_t* traverse,
                      size_t cap, size_t* n) {
  if (!s || !ref || !n) return BSG_EINVAL;
  bs::Ref r;
  std::memcpy(r.data(), ref, 32);
  std::vector<bs::split::ProtectPair> pairs;
  bs::Status st = bs::split::Protect(s->st.get(), r, &pairs);
  if (!st.ok()) return st.code;
  *n = pairs.size();
  for (size_t i = 0; i < pairs.size() && i < cap; ++i) {
    if (refs) std::memcpy(refs + 32 * i, pairs[i].ref.data(), 32);
    if (traverse) traverse[i] = pairs[i].traverse ? 1 : 0;
  }
  return BSG_OK;
}

size_t bsg_store_list_from(bsg_store* s, const uint8_t start[32], uint8_t* refs, size_t cap) {
  if (!s || !start) return 0;
  bs::Ref st;
  std::memcpy(st.data(), start, 32);
  size_t k = 0;
  s->st->ListRefs(st, [&](const bs::Ref& r) {
    if (k < cap && refs) std::memcpy(refs + 32 * k, r.data(), 32);
    ++k;
    return bs::Status::Ok();
  });
  return k;
}

size_t bsg_store_list(bsg_store* s, uint8_t* refs, size_t cap) {
  if (!s) return 0;
  size_t k = 0;
  s->st->ListRefs(bs::Zero, [&](const bs::Ref& r) {
    if (k < cap && refs) std::memcpy(refs + 32 * k, r.data(), 32);
    ++k;
    return bs::Status::Ok();
  });
  return k;  // note: bs::Zero itself is never listed (ListRefs starts after `start`)
}

bsg_writer* bsg_writer_new(int device, bsg_store* s, const bsg_params* params, size_t tile,
                           int* err) {
  int dummy;
  if (!err) err = &dummy;
  if (!s) {
    *err = BSG_EINVAL;
    return nullptr;
  }
  bs::split::Options o;
  if (params) {
    o.bits = params->split_bits;
    o.min_size = (int)params->min_size;
    o.fanout = params->fanout;
  }
  o.device = device;
  o.tile = tile;
  bs::Status st;
  auto w = bs::split::Writer::New(s->st.get(), o, &st);
  if (!w) {
    *err = st.code;
    return nullptr;
  }
  *err = BSG_OK;
  return new bsg_writer{std::move(w)};
}

int bsg_writer_write(bsg_writer* w, const uint8_t* p, size_t n) {
  if (!w) return BSG_EINVAL;
  return w->w->Write(p, n).code;
}
int bsg_writer_close(bsg_writer* w) { return w ? w->w->Close().code : BSG_EINVAL; }
int bsg_writer_set_stream_base(bsg_writer* w, uint64_t base) {
  return w ? w->w->SetStreamBase(base).code : BSG_EINVAL;
}
int bsg_writer_root(const bsg_writer* w, uint8_t out[32]) {
  if (!w || !out) return BSG_EINVAL;
  std::memcpy(out, w->w->Root().data(), 32);
  return BSG_OK;
}
int bsg_writer_timings(const bsg_writer* w, double out[7]) {
  if (!w || !out) return BSG_EINVAL;
  w->w->Timings(out);
  return BSG_OK;
}
void bsg_writer_free(bsg_writer* w) { delete w; }

bsg_reader* bsg_reader_new(bsg_store* s, const uint8_t root[32], int* err) {
  return bsg_reader_open(s, root, 0, 0, err);
}

bsg_reader* bsg_reader_open(bsg_store* s, const uint8_t root[32], int flags, int device,
                            int* err) {
  int dummy;
  if (!err) err = &dummy;
  if (!s || !root) {
    *err = BSG_EINVAL;
    return nullptr;
  }
  bs::Ref r;
  std::memcpy(r.data(), root, 32);
  bs::Status st;
  auto rd = bs::split::Reader::New(s->st.get(), r, &st, (flags & BSG_READER_VERIFY) != 0, device);
  if (!rd) {
    *err = st.code;
    return nullptr;
  }
  *err = BSG_OK;
  return new bsg_reader{std::move(rd)};
}

int64_t bsg_reader_read(bsg_reader* r, uint8_t* buf, size_t n) {
  if (!r || (!buf && n)) return BSG_EINVAL;
  size_t got = 0;
  bool eof = false;
  bs::Status st = r->r->Read(buf, n, &got, &eof);
  if (!st.ok()) return st.code;
  return (int64_t)got;
}
int64_t bsg_reader_seek(bsg_reader* r, int64_t off, int whence) {
  return r ? (int64_t)r->r->Seek(off, whence) : BSG_EINVAL;
}
uint64_t bsg_reader_size(const bsg_reader* r) { return r ? r->r->Size() : 0; }
int bsg_reader_stats(const bsg_reader* r, uint64_t out[4]) {
  if (!r || !out) return BSG_EINVAL;
  r->r->Stats(out);
  return BSG_OK;
}
void bsg_reader_free(bsg_reader* r) { delete r; }

}  // extern "C"
