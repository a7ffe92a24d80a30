// bs_filestore.cpp — bs::FileStore, the host mirror of store/file (reference
// store/file/file.go:20-154): one file per blob at <root>/blobs/<hex[:2]>/<hex[:4]>/<hex>.
// Put's ref comes from the GPU (GpuHasher -> bsg_sha256_batch) or, through PutWithRef, from the
// chunk records the split kernels already produced, so an ingest never hashes a blob twice.
// Anchor-map files (file.go:156-230) are outside the hot path and not mirrored.
#include <dirent.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstring>

#include "../../include/bs_split.hpp"

namespace bs {

namespace {

Status errno_status(const std::string& what) {
  return Status::Err(kIO, what + ": " + std::strerror(errno));
}

// os.MkdirAll(dir, 0755)
Status mkdir_all(const std::string& dir) {
  if (dir.empty()) return Status::Ok();
  struct stat sb;
  if (::stat(dir.c_str(), &sb) == 0) {
    if (S_ISDIR(sb.st_mode)) return Status::Ok();
    errno = ENOTDIR;
    return errno_status("ensuring path " + dir + " exists");
  }
  const size_t slash = dir.find_last_of('/');
  if (slash != std::string::npos && slash > 0) {
    Status s = mkdir_all(dir.substr(0, slash));
    if (!s.ok()) return s;
  }
  if (::mkdir(dir.c_str(), 0755) != 0 && errno != EEXIST)
    return errno_status("ensuring path " + dir + " exists");
  return Status::Ok();
}

// ioutil.ReadDir: entries sorted by name, with an is-directory flag; "." and ".." skipped.
struct Entry {
  std::string name;
  bool dir;
};
Status read_dir(const std::string& path, std::vector<Entry>* out) {
  out->clear();
  DIR* d = ::opendir(path.c_str());
  if (!d) return errno_status("reading dir " + path);
  while (struct dirent* e = ::readdir(d)) {
    const std::string name = e->d_name;
    if (name == "." || name == "..") continue;
    bool isdir;
    if (e->d_type == DT_DIR || e->d_type == DT_REG) {
      isdir = e->d_type == DT_DIR;
    } else {  // DT_UNKNOWN on some filesystems
      struct stat sb;
      isdir = ::stat((path + "/" + name).c_str(), &sb) == 0 && S_ISDIR(sb.st_mode);
    }
    out->push_back({name, isdir});
  }
  ::closedir(d);
  std::sort(out->begin(), out->end(), [](const Entry& a, const Entry& b) { return a.name < b.name; });
  return Status::Ok();
}

bool is_hex(const std::string& s) {
  return !s.empty() && std::all_of(s.begin(), s.end(), [](char c) {
    return (c >= '0' && c <= '9') || (c >= 'a' && c <= 'f') || (c >= 'A' && c <= 'F');
  });
}

}  // namespace

bool RefFromHex(const std::string& hex, Ref* out) {
  if (hex.size() != 64 || !is_hex(hex)) return false;
  auto nib = [](char c) -> int {
    return c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10;
  };
  for (int i = 0; i < 32; ++i) (*out)[i] = (uint8_t)(nib(hex[2 * i]) << 4 | nib(hex[2 * i + 1]));
  return true;
}

std::string FileStore::BlobPath(const Ref& ref) const {  // file.go:33-40
  const std::string h = RefString(ref);
  return root_ + "/blobs/" + h.substr(0, 2) + "/" + h.substr(0, 4) + "/" + h;
}

FileStore::~FileStore() {
  const Status s0 = FlushAll();  // group 0's error, which FlushAll reports (and clears)
  if (!s0.ok())
    std::fprintf(stderr, "bs::FileStore(%s): unreported write error (group 0): %s\n",
                 root_.c_str(), s0.msg.c_str());
  {
    std::lock_guard<std::mutex> g(wb_mu_);
    wb_stop_ = true;
    // errors no caller has collected with Flush: nobody is left to return them to
    for (const auto& kv : groups_)
      if (!kv.second.err.ok())
        std::fprintf(stderr, "bs::FileStore(%s): unreported write error (group %llu): %s\n",
                     root_.c_str(), (unsigned long long)kv.first, kv.second.err.msg.c_str());
  }
  wb_cv_.notify_all();
  for (std::thread& t : wb_threads_) t.join();
}

Status FileStore::MkdirFor(const std::string& path) {
  const std::string dir = path.substr(0, path.find_last_of('/'));
  const std::string hhhh = dir.substr(dir.size() - 4);
  uint32_t k = 0;
  for (char c : hhhh) k = k << 4 | (uint32_t)(c <= '9' ? c - '0' : (c | 0x20) - 'a' + 10);
  {
    std::lock_guard<std::mutex> g(dir_mu_);
    if (dirs_made_[k & 0xffff]) return Status::Ok();
  }
  Status s = mkdir_all(dir);
  if (!s.ok()) return s;
  std::lock_guard<std::mutex> g(dir_mu_);
  dirs_made_[k & 0xffff] = true;
  return Status::Ok();
}

uint64_t FileStore::OpenGroup() {
  std::lock_guard<std::mutex> g(wb_mu_);
  const uint64_t id = next_group_++;
  groups_[id] = Group{};
  return id;
}

void FileStore::CloseGroup(uint64_t group) {
  if (group == 0) return;
  std::lock_guard<std::mutex> g(wb_mu_);
  auto it = groups_.find(group);
  if (it == groups_.end()) return;
  if (it->second.outstanding == 0 && it->second.err.ok()) {
    groups_.erase(it);
  } else {
    it->second.closed = true;  // erased by the worker that writes its last blob
  }
}

void FileStore::SetWriteBehindLimit(uint64_t bytes) {
  std::lock_guard<std::mutex> g(wb_mu_);
  wb_limit_ = std::max<uint64_t>(1, bytes);
}

void FileStore::Attach(Pending& p, uint64_t group) {
  if (std::find(p.groups.begin(), p.groups.end(), group) != p.groups.end()) return;
  p.groups.push_back(group);
  groups_[group].outstanding++;
}

Status FileStore::PutBlob(const Ref& ref, const Blob& b, bool* added, uint64_t group) {
  if (added) *added = false;
  std::unique_lock<std::mutex> g(wb_mu_);
  if (!groups_.count(group)) return Status::Err(BSG_EINVAL, "unknown write group");
  auto it = wb_pending_.find(ref);
  if (it != wb_pending_.end()) {  // queued by someone: this group waits for that write too
    Attach(it->second, group);
    return Status::Ok();
  }
  if (wb_threads_.empty())
    for (int i = 0; i < kWriterThreads; ++i) wb_threads_.emplace_back([this] { Worker(); });
  // bounded: wait for the writers while the limit's worth of bytes is pending
  wb_done_cv_.wait(g, [&] { return wb_bytes_ < wb_limit_; });
  // another caller may have queued the same blob while this one waited
  it = wb_pending_.find(ref);
  if (it != wb_pending_.end()) {
    Attach(it->second, group);
    return Status::Ok();
  }
  Pending& p = wb_pending_[ref];
  p.blob = b;
  Attach(p, group);
  wb_bytes_ += b.size;
  wb_queue_.push_back(ref);
  if (added) *added = true;
  g.unlock();
  wb_cv_.notify_one();
  return Status::Ok();
}

void FileStore::Worker() {
  for (;;) {
    Ref ref;
    Blob blob;
    {
      std::unique_lock<std::mutex> g(wb_mu_);
      wb_cv_.wait(g, [&] { return wb_stop_ || !wb_queue_.empty(); });
      if (wb_queue_.empty()) return;  // stopping
      ref = wb_queue_.front();
      wb_queue_.pop_front();
      blob = wb_pending_.at(ref).blob;  // the entry stays (Get serves it) until written
    }
    bool added = false;
    Status s = PutWithRef(ref, blob.bytes(), blob.size, &added);
    {
      std::lock_guard<std::mutex> g(wb_mu_);
      auto it = wb_pending_.find(ref);
      for (uint64_t id : it->second.groups) {
        Group& gr = groups_[id];
        if (!s.ok() && gr.err.ok()) gr.err = s;
        if (--gr.outstanding == 0 && gr.closed && gr.err.ok()) groups_.erase(id);
      }
      wb_pending_.erase(it);
      wb_bytes_ -= blob.size;
    }
    wb_done_cv_.notify_all();
  }
}

Status FileStore::Flush(uint64_t group) {
  std::unique_lock<std::mutex> g(wb_mu_);
  auto it = groups_.find(group);
  if (it == groups_.end()) return Status::Err(BSG_EINVAL, "unknown write group");
  // (a closed group with nothing outstanding and no error is erased by the last worker)
  wb_done_cv_.wait(g, [&] {
    auto i = groups_.find(group);
    return i == groups_.end() || i->second.outstanding == 0;
  });
  it = groups_.find(group);
  if (it == groups_.end()) return Status::Ok();
  Status s = it->second.err;
  it->second.err = Status::Ok();  // reported once
  if (it->second.closed && group != 0) groups_.erase(it);
  return s;
}

Status FileStore::FlushAll() {
  {
    std::unique_lock<std::mutex> g(wb_mu_);
    wb_done_cv_.wait(g, [&] { return wb_pending_.empty(); });
  }
  return Flush(0);
}

Status FileStore::GetBlob(const Ref& ref, Blob* out) {
  {
    std::lock_guard<std::mutex> g(wb_mu_);
    auto it = wb_pending_.find(ref);
    if (it != wb_pending_.end()) {
      *out = it->second.blob;
      return Status::Ok();
    }
  }
  return Store::GetBlob(ref, out);
}

Status FileStore::Get(const Ref& ref, std::vector<uint8_t>* out) {  // file.go:42-50
  {
    std::lock_guard<std::mutex> g(wb_mu_);
    auto it = wb_pending_.find(ref);
    if (it != wb_pending_.end()) {  // accepted by PutBlob, not written yet
      const Blob& b = it->second.blob;
      out->assign(b.bytes(), b.bytes() + b.size);
      return Status::Ok();
    }
  }
  const std::string path = BlobPath(ref);
  const int fd = ::open(path.c_str(), O_RDONLY);
  if (fd < 0) {
    if (errno == ENOENT) return Status::Err(kNotFound, "not found");
    return errno_status("opening " + path);
  }
  out->clear();
  struct stat sb;
  if (::fstat(fd, &sb) == 0 && sb.st_size > 0) out->reserve((size_t)sb.st_size);
  uint8_t buf[1 << 16];
  for (;;) {
    const ssize_t k = ::read(fd, buf, sizeof buf);
    if (k < 0) {
      if (errno == EINTR) continue;
      Status s = errno_status("opening " + path);
      ::close(fd);
      return s;
    }
    if (k == 0) break;
    out->insert(out->end(), buf, buf + k);
  }
  ::close(fd);
  return Status::Ok();
}

Status FileStore::Put(const uint8_t* data, size_t n, Ref* ref, bool* added) {  // file.go:52-76
  Ref r;
  Status s = hasher_.Sum(data, n, &r);
  if (!s.ok()) return s;
  if (ref) *ref = r;
  return PutWithRef(r, data, n, added);
}

Status FileStore::PutWithRef(const Ref& ref, const uint8_t* data, size_t n, bool* added) {
  if (added) *added = false;
  const std::string path = BlobPath(ref);
  Status s = MkdirFor(path);
  if (!s.ok()) return s;
  const int fd = ::open(path.c_str(), O_WRONLY | O_CREAT | O_EXCL, 0644);
  if (fd < 0) {
    if (errno == EEXIST) return Status::Ok();  // already present: (ref, false, nil)
    return errno_status("creating " + path);
  }
  size_t done = 0;
  while (done < n) {
    const ssize_t k = ::write(fd, data + done, n - done);
    if (k < 0) {
      if (errno == EINTR) continue;
      s = errno_status("writing data to " + path);
      ::close(fd);
      return s;
    }
    done += (size_t)k;
  }
  if (::close(fd) != 0) return errno_status("writing data to " + path);
  if (added) *added = true;
  return Status::Ok();
}

// file.go:79-154: walk blobs/<2>/<4>/<64> in name order, starting after `start`.
Status FileStore::ListRefs(const Ref& start, const std::function<Status(const Ref&)>& f) {
  Status s = FlushAll();  // blobs accepted by PutBlob are listed once written
  if (!s.ok()) return s;
  const std::string blobroot = root_ + "/blobs";
  s = mkdir_all(blobroot);
  if (!s.ok()) return s;
  std::vector<Entry> top, mid, blobs;
  s = read_dir(blobroot, &top);
  if (!s.ok()) return s;
  const std::string sh = RefString(start);
  auto ti = std::lower_bound(top.begin(), top.end(), sh.substr(0, 2),
                             [](const Entry& e, const std::string& k) { return e.name < k; });
  for (; ti != top.end(); ++ti) {
    if (!ti->dir || ti->name.size() != 2 || !is_hex(ti->name)) continue;
    const std::string tdir = blobroot + "/" + ti->name;
    s = read_dir(tdir, &mid);
    if (!s.ok()) return s;
    auto mi = std::lower_bound(mid.begin(), mid.end(), sh.substr(0, 4),
                               [](const Entry& e, const std::string& k) { return e.name < k; });
    for (; mi != mid.end(); ++mi) {
      if (!mi->dir || mi->name.size() != 4 || !is_hex(mi->name)) continue;
      s = read_dir(tdir + "/" + mi->name, &blobs);
      if (!s.ok()) return s;
      auto bi = std::upper_bound(blobs.begin(), blobs.end(), sh,
                                 [](const std::string& k, const Entry& e) { return k < e.name; });
      for (; bi != blobs.end(); ++bi) {
        if (bi->dir) continue;
        Ref r;
        if (!RefFromHex(bi->name, &r)) continue;
        s = f(r);
        if (!s.ok()) return s;
      }
    }
  }
  return Status::Ok();
}

}  // namespace bs
