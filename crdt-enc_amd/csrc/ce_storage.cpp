// ce_storage.cpp -- Storage plugin (crdt-enc/src/storage.rs:8-43) with the crdt-enc-tokio
// local-dir layout (crdt-enc-tokio/src/lib.rs), content naming (SHA3-256 + BASE32_NOPAD,
// tokio lib.rs:403-432), UUID text forms and the VersionBytesBuf framing helpers
// (crdt-enc/src/utils/version_bytes.rs:245-309).
#include <dirent.h>
#include <dlfcn.h>
#include <errno.h>
#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdio>
#include <deque>
#include <mutex>
#include <string>
#include <thread>
#include <unordered_map>
#include <unordered_set>

#include "ce_internal.h"

namespace ce {

std::string uuid_to_string(const Uuid& u) {
  static const char* hx = "0123456789abcdef";
  std::string s;
  s.reserve(36);
  for (int i = 0; i < 16; i++) {
    if (i == 4 || i == 6 || i == 8 || i == 10) s.push_back('-');
    s.push_back(hx[u[i] >> 4]);
    s.push_back(hx[u[i] & 15]);
  }
  return s;
}

static int hexv(char c) {
  if (c >= '0' && c <= '9') return c - '0';
  if (c >= 'a' && c <= 'f') return c - 'a' + 10;
  if (c >= 'A' && c <= 'F') return c - 'A' + 10;
  return -1;
}

// uuid 1.x Uuid::from_str: simple (32 hex), hyphenated (8-4-4-4-12), braced, urn:uuid:
bool uuid_parse(const std::string& in, Uuid* out) {
  std::string s = in;
  if (s.size() == 45 && s.compare(0, 9, "urn:uuid:") == 0) s = s.substr(9);
  else if (s.size() == 38 && s.front() == '{' && s.back() == '}') s = s.substr(1, 36);
  std::string h;
  if (s.size() == 36) {
    for (size_t i = 0; i < 36; i++) {
      if (i == 8 || i == 13 || i == 18 || i == 23) {
        if (s[i] != '-') return false;
      } else h.push_back(s[i]);
    }
  } else if (s.size() == 32) h = s;
  else return false;
  for (int i = 0; i < 16; i++) {
    int a = hexv(h[2 * i]), b = hexv(h[2 * i + 1]);
    if (a < 0 || b < 0) return false;
    (*out)[i] = (uint8_t)(a * 16 + b);
  }
  return true;
}

Uuid uuid_v4() {
  Uuid u;
  os_random(u.data(), 16);
  u[6] = (u[6] & 0x0f) | 0x40;
  u[8] = (u[8] & 0x3f) | 0x80;
  return u;
}

// ---- SHA3-256 (FIPS 202): Keccak-f[1600] with every index compile-time (fully unrolled) ----
static inline uint64_t rotl64(uint64_t x, int n) { return n ? (x << n) | (x >> (64 - n)) : x; }

namespace {
constexpr uint64_t kRC[24] = {
    0x0000000000000001ull, 0x0000000000008082ull, 0x800000000000808aull, 0x8000000080008000ull,
    0x000000000000808bull, 0x0000000080000001ull, 0x8000000080008081ull, 0x8000000000008009ull,
    0x000000000000008aull, 0x0000000000000088ull, 0x0000000080008009ull, 0x000000008000000aull,
    0x000000008000808bull, 0x800000000000008bull, 0x8000000000008089ull, 0x8000000000008003ull,
    0x8000000000008002ull, 0x8000000000000080ull, 0x000000000000800aull, 0x800000008000000aull,
    0x8000000080008081ull, 0x8000000000008080ull, 0x0000000080000001ull, 0x8000000080008008ull};
// rho offsets r[x][y] (lane x + 5y)
constexpr int kRho[25] = {0, 1, 62, 28, 27, 36, 44, 6, 55, 20, 3, 10, 43,
                          25, 39, 41, 45, 15, 21, 8, 18, 2, 61, 56, 14};
}  // namespace

static void keccakf(uint64_t s[25]);
void keccakf_portable(uint64_t s[25]) { keccakf(s); }  // (ce_sha3x8.cpp: message tails)

static void keccakf(uint64_t s[25]) {
  for (int r = 0; r < 24; r++) {
    uint64_t c[5], b[25];
#pragma clang loop unroll(full)
    for (int x = 0; x < 5; x++) c[x] = s[x] ^ s[x + 5] ^ s[x + 10] ^ s[x + 15] ^ s[x + 20];
    // theta + rho + pi: B[y, 2x+3y] = rot(A[x, y] ^ D[x], r[x, y])
#pragma clang loop unroll(full)
    for (int x = 0; x < 5; x++) {
      const uint64_t d = c[(x + 4) % 5] ^ rotl64(c[(x + 1) % 5], 1);
#pragma clang loop unroll(full)
      for (int y = 0; y < 5; y++) b[y + 5 * ((2 * x + 3 * y) % 5)] = rotl64(s[x + 5 * y] ^ d, kRho[x + 5 * y]);
    }
    // chi + iota
#pragma clang loop unroll(full)
    for (int y = 0; y < 25; y += 5) {
#pragma clang loop unroll(full)
      for (int x = 0; x < 5; x++) s[y + x] = b[y + x] ^ (~b[y + (x + 1) % 5] & b[y + (x + 2) % 5]);
    }
    s[0] ^= kRC[r];
  }
}

// OpenSSL's EVP SHA3-256 (AVX2 Keccak, ~2x this file's portable one) when libcrypto.so.3 is
// present -- resolved once with dlopen, so the library has no link-time dependency on it.
namespace {
struct EvpSha3 {
  using new_t = void* (*)();
  using free_t = void (*)(void*);
  using md_t = const void* (*)();
  using init_t = int (*)(void*, const void*, void*);
  using upd_t = int (*)(void*, const void*, size_t);
  using fin_t = int (*)(void*, unsigned char*, unsigned int*);
  new_t ctx_new = nullptr;
  free_t ctx_free = nullptr;
  md_t sha3 = nullptr;
  init_t init = nullptr;
  upd_t update = nullptr;
  fin_t final = nullptr;
  bool ok = false;
  EvpSha3() {
    if (std::getenv("CE_NO_OPENSSL")) return;
    void* h = dlopen("libcrypto.so.3", RTLD_NOW | RTLD_LOCAL);
    if (!h) return;
    ctx_new = (new_t)dlsym(h, "EVP_MD_CTX_new");
    ctx_free = (free_t)dlsym(h, "EVP_MD_CTX_free");
    sha3 = (md_t)dlsym(h, "EVP_sha3_256");
    init = (init_t)dlsym(h, "EVP_DigestInit_ex");
    update = (upd_t)dlsym(h, "EVP_DigestUpdate");
    final = (fin_t)dlsym(h, "EVP_DigestFinal_ex");
    ok = ctx_new && ctx_free && sha3 && init && update && final;
  }
  bool digest(const uint8_t* msg, size_t len, uint8_t out[32]) const {
    if (!ok) return false;
    void* c = ctx_new();
    if (!c) return false;
    unsigned int n = 0;
    const bool good = init(c, sha3(), nullptr) == 1 && update(c, msg, len) == 1 && final(c, out, &n) == 1 && n == 32;
    ctx_free(c);
    return good;
  }
};
}  // namespace

void sha3_256(const uint8_t* msg, size_t len, uint8_t out[32]) {
  static const EvpSha3 evp;
  if (len >= 4096 && evp.digest(msg, len, out)) return;
  uint64_t st[25] = {0};
  const size_t rate = 136;
  auto absorb = [&](const uint8_t* b) {
    for (size_t i = 0; i < rate / 8; i++) {
      uint64_t w;
      std::memcpy(&w, b + 8 * i, 8);
      st[i] ^= w;
    }
    keccakf(st);
  };
  while (len >= rate) {
    absorb(msg);
    msg += rate;
    len -= rate;
  }
  uint8_t last[136] = {0};
  std::memcpy(last, msg, len);
  last[len] ^= 0x06;
  last[rate - 1] ^= 0x80;
  absorb(last);
  std::memcpy(out, st, 32);
}

std::string base32_nopad(const uint8_t* in, size_t len) {
  static const char* A = "ABCDEFGHIJKLMNOPQRSTUVWXYZ234567";
  std::string s;
  uint64_t buf = 0;
  int bits = 0;
  for (size_t i = 0; i < len; i++) {
    buf = (buf << 8) | in[i];
    bits += 8;
    while (bits >= 5) {
      s.push_back(A[(buf >> (bits - 5)) & 31]);
      bits -= 5;
    }
  }
  if (bits) s.push_back(A[(buf << (5 - bits)) & 31]);
  return s;
}

}  // namespace ce

using namespace ce;

static bool read_file(const std::string& path, std::vector<uint8_t>* out, bool* missing) {
  *missing = false;
  int fd = ::open(path.c_str(), O_RDONLY | O_CLOEXEC);
  if (fd < 0) {
    *missing = errno == ENOENT;
    return false;
  }
  struct stat st;
  if (fstat(fd, &st) != 0) { ::close(fd); return false; }
  out->resize((size_t)st.st_size);
  size_t got = 0;
  while (got < out->size()) {
    ssize_t r = ::read(fd, out->data() + got, out->size() - got);
    if (r <= 0) { ::close(fd); return false; }
    got += (size_t)r;
  }
  ::close(fd);
  return true;
}

// tokio write_file_inner (lib.rs:326-346): create_new (or truncate), write, flush, fsync
static int write_file(const std::string& path, const uint8_t* d, size_t n, bool create_new) {
  int fl = O_WRONLY | O_CLOEXEC | O_CREAT | (create_new ? O_EXCL : O_TRUNC);
  int fd = ::open(path.c_str(), fl, 0644);
  if (fd < 0) return CE_ERR_IO;
  size_t put = 0;
  while (put < n) {
    ssize_t w = ::write(fd, d + put, n - put);
    if (w <= 0) { ::close(fd); return CE_ERR_IO; }
    put += (size_t)w;
  }
  if (fsync(fd) != 0) { ::close(fd); return CE_ERR_IO; }
  ::close(fd);
  return CE_OK;
}

static int mkdirs(const std::string& p) {
  std::string cur;
  for (size_t i = 0; i < p.size(); i++) {
    cur.push_back(p[i]);
    if ((p[i] == '/' && i > 0) || i + 1 == p.size()) {
      if (::mkdir(cur.c_str(), 0755) != 0 && errno != EEXIST) return CE_ERR_IO;
    }
  }
  return CE_OK;
}

static int list_dir(const std::string& path, bool want_files, std::vector<std::string>* out) {
  DIR* d = opendir(path.c_str());
  if (!d) return errno == ENOENT ? CE_OK : CE_ERR_IO;  // read_dir_optional: NotFound = empty
  while (struct dirent* e = readdir(d)) {
    std::string n = e->d_name;
    if (n == "." || n == "..") continue;
    struct stat st;
    if (stat((path + "/" + n).c_str(), &st) != 0) continue;
    if (want_files ? S_ISREG(st.st_mode) : S_ISDIR(st.st_mode)) out->push_back(n);
  }
  closedir(d);
  return CE_OK;
}

static int remove_optional(const std::string& p) {
  if (::unlink(p.c_str()) == 0 || errno == ENOENT) return CE_OK;
  return CE_ERR_IO;
}

static int set_buf(ce_buf* b, const void* d, size_t n) {
  b->data = (uint8_t*)malloc(n ? n : 1);
  if (!b->data) return CE_ERR_INVALID_ARG;
  if (n) std::memcpy(b->data, d, n);
  b->len = n;
  return CE_OK;
}

namespace ce {
// used by the core
int storage_load_ops_vec(ce_storage* s, const std::vector<Uuid>& actors,
                         const std::vector<uint64_t>& first, std::vector<uint8_t>* blob,
                         std::vector<uint64_t>* offs, std::vector<uint32_t>* aidx,
                         std::vector<uint64_t>* vers) {
  offs->assign(1, 0);
  for (size_t a = 0; a < actors.size(); a++) {
    const std::string dir = s->remote + "/ops/" + uuid_to_string(actors[a]);
    // tokio load_ops (lib.rs:249-270): read first, first+1, ... until NotFound
    for (uint64_t v = first[a];; v++) {
      std::vector<uint8_t> f;
      bool missing;
      if (!read_file(dir + "/" + std::to_string(v), &f, &missing)) {
        if (missing) break;
        return CE_ERR_IO;
      }
      blob->insert(blob->end(), f.begin(), f.end());
      offs->push_back(blob->size());
      aidx->push_back((uint32_t)a);
      vers->push_back(v);
    }
  }
  return CE_OK;
}
int storage_list_op_actors_vec(ce_storage* s, std::vector<Uuid>* out) {
  std::vector<std::string> names;
  int rc = list_dir(s->remote + "/ops", false, &names);
  if (rc) return rc;
  for (auto& n : names) {
    Uuid u;
    if (!uuid_parse(n, &u)) return CE_ERR_IO;  // "error converting actor dir string into uuid"
    out->push_back(u);
  }
  return CE_OK;
}
int storage_list_states_vec(ce_storage* s, std::vector<std::string>* out) {
  return list_dir(s->remote + "/states", true, out);
}
int storage_read_state(ce_storage* s, const std::string& name, std::vector<uint8_t>* out) {
  bool missing;
  return read_file(s->remote + "/states/" + name, out, &missing) ? CE_OK : CE_ERR_IO;
}
int storage_store_content(ce_storage* s, const char* sub, const uint8_t* d, size_t n,
                          std::string* name) {
  uint8_t h[32];
  sha3_256(d, n, h);
  *name = base32_nopad(h, 32);
  const std::string dir = s->remote + "/" + sub;
  if (mkdirs(dir)) return CE_ERR_IO;
  return write_file(dir + "/" + *name, d, n, true);
}
int storage_remove_state(ce_storage* s, const std::string& name) {
  return remove_optional(s->remote + "/states/" + name);
}
int storage_store_op(ce_storage* s, const Uuid& actor, uint64_t version, const uint8_t* d,
                     size_t n) {
  const std::string dir = s->remote + "/ops/" + uuid_to_string(actor);
  if (mkdirs(dir)) return CE_ERR_IO;
  return write_file(dir + "/" + std::to_string(version), d, n, true);
}
int storage_remove_op(ce_storage* s, const Uuid& actor, uint64_t version) {
  return remove_optional(s->remote + "/ops/" + uuid_to_string(actor) + "/" + std::to_string(version));
}
int storage_load_local_meta(ce_storage* s, std::vector<uint8_t>* out, bool* missing) {
  if (read_file(s->local + "/meta-data.msgpack", out, missing)) return CE_OK;
  return *missing ? CE_OK : CE_ERR_IO;
}
int storage_store_local_meta(ce_storage* s, const uint8_t* d, size_t n) {
  if (mkdirs(s->local)) return CE_ERR_IO;
  return write_file(s->local + "/meta-data.msgpack", d, n, false);
}
ce_storage* storage_new(const std::string& local, const std::string& remote) {
  ce_storage* s = new ce_storage();
  s->local = local;
  s->remote = remote;
  return s;
}
}  // namespace ce

// One native worker for ce_content_name_async: the caller's thread only queues the job (no
// Python thread, hence no interpreter-lock hand-offs between the caller and the hash).  The
// worker is detached and lives for the process.
namespace {
struct NameWorker {
  struct Job {
    uint64_t id;
    const uint8_t* data;
    size_t len;
  };
  std::mutex mu;
  std::condition_variable cv_job, cv_done;
  std::deque<Job> q;
  std::unordered_map<uint64_t, std::string> done;
  std::unordered_set<uint64_t> pending;  // queued or hashing
  uint64_t next = 1;
  bool started = false;
  void run() {
    std::unique_lock<std::mutex> lk(mu);
    for (;;) {
      cv_job.wait(lk, [&] { return !q.empty(); });
      const Job j = q.front();
      q.pop_front();
      lk.unlock();
      uint8_t h[32];
      sha3_256(j.data, j.len, h);
      std::string nm = base32_nopad(h, 32);
      lk.lock();
      pending.erase(j.id);
      done.emplace(j.id, std::move(nm));
      cv_done.notify_all();
    }
  }
};
NameWorker& name_worker() {
  static NameWorker* w = new NameWorker;  // never destroyed: the detached worker may still run
  return *w;
}
}  // namespace

extern "C" {

int ce_storage_open(const char* local_path, const char* remote_path, ce_storage** out) {
  if (!local_path || !remote_path || !out) return CE_ERR_INVALID_ARG;
  // Storage::new: both paths must be absolute (tokio lib.rs:29-39)
  if (local_path[0] != '/' || remote_path[0] != '/') return CE_ERR_INVALID_ARG;
  *out = storage_new(local_path, remote_path);
  return CE_OK;
}

void ce_storage_close(ce_storage* s) { delete s; }

int ce_storage_list_op_actors(ce_storage* s, ce_buf* out) {
  if (!s || !out) return CE_ERR_INVALID_ARG;
  std::vector<Uuid> a;
  int rc = storage_list_op_actors_vec(s, &a);
  if (rc) return rc;
  return set_buf(out, a.data(), a.size() * 16);
}

int ce_storage_load_ops(ce_storage* s, const uint8_t* actors, const uint64_t* first, uint32_t m,
                        ce_buf* blob, ce_buf* offs, ce_buf* actor_idx, ce_buf* versions) {
  if (!s || (m && (!actors || !first)) || !blob || !offs || !actor_idx || !versions)
    return CE_ERR_INVALID_ARG;
  std::vector<Uuid> av(m);
  for (uint32_t i = 0; i < m; i++) std::memcpy(av[i].data(), actors + 16 * i, 16);
  std::vector<uint64_t> fv(first, first + m), o, ver;
  std::vector<uint8_t> b;
  std::vector<uint32_t> ai;
  int rc = storage_load_ops_vec(s, av, fv, &b, &o, &ai, &ver);
  if (rc) return rc;
  set_buf(blob, b.data(), b.size());
  set_buf(offs, o.data(), o.size() * 8);
  set_buf(actor_idx, ai.data(), ai.size() * 4);
  set_buf(versions, ver.data(), ver.size() * 8);
  return CE_OK;
}

int ce_storage_store_ops(ce_storage* s, const uint8_t actor[16], uint64_t version,
                         const uint8_t* data, size_t len) {
  if (!s || !actor || (len && !data)) return CE_ERR_INVALID_ARG;
  Uuid a;
  std::memcpy(a.data(), actor, 16);
  return storage_store_op(s, a, version, data, len);
}

int ce_storage_remove_ops(ce_storage* s, const uint8_t* actors, const uint64_t* versions,
                          uint32_t m) {
  if (!s || (m && (!actors || !versions))) return CE_ERR_INVALID_ARG;
  for (uint32_t i = 0; i < m; i++) {
    Uuid a;
    std::memcpy(a.data(), actors + 16 * i, 16);
    int rc = storage_remove_op(s, a, versions[i]);
    if (rc) return rc;
  }
  return CE_OK;
}

int ce_storage_list_state_names(ce_storage* s, ce_buf* out) {
  if (!s || !out) return CE_ERR_INVALID_ARG;
  std::vector<std::string> names;
  int rc = storage_list_states_vec(s, &names);
  if (rc) return rc;
  std::string j;
  for (auto& n : names) { j += n; j.push_back('\0'); }
  return set_buf(out, j.data(), j.size());
}

int ce_storage_store_state(ce_storage* s, const uint8_t* data, size_t len, char name_out[64]) {
  if (!s || (len && !data)) return CE_ERR_INVALID_ARG;
  std::string name;
  int rc = storage_store_content(s, "states", data, len, &name);
  if (rc) return rc;
  if (name_out) std::snprintf(name_out, 64, "%s", name.c_str());
  return CE_OK;
}

int ce_storage_load_state(ce_storage* s, const char* name, ce_buf* out) {
  if (!s || !name || !out) return CE_ERR_INVALID_ARG;
  std::vector<uint8_t> d;
  int rc = storage_read_state(s, name, &d);
  if (rc) return rc;
  return set_buf(out, d.data(), d.size());
}

int ce_storage_remove_state(ce_storage* s, const char* name) {
  if (!s || !name) return CE_ERR_INVALID_ARG;
  return storage_remove_state(s, name);
}

int ce_content_name(const uint8_t* data, size_t len, char name_out[64]) {
  if ((len && !data) || !name_out) return CE_ERR_INVALID_ARG;
  uint8_t h[32];
  sha3_256(data, len, h);
  std::snprintf(name_out, 64, "%s", base32_nopad(h, 32).c_str());
  return CE_OK;
}

int ce_content_name_async(const uint8_t* data, size_t len, uint64_t* ticket) {
  if ((len && !data) || !ticket) return CE_ERR_INVALID_ARG;
  NameWorker& w = name_worker();
  std::lock_guard<std::mutex> g(w.mu);
  if (!w.started) {
    std::thread([&w] { w.run(); }).detach();
    w.started = true;
  }
  *ticket = w.next++;
  w.pending.insert(*ticket);
  w.q.push_back({*ticket, data, len});
  w.cv_job.notify_one();
  return CE_OK;
}

int ce_content_name_wait(uint64_t ticket, char name_out[64]) {
  if (!name_out) return CE_ERR_INVALID_ARG;
  NameWorker& w = name_worker();
  std::unique_lock<std::mutex> lk(w.mu);
  auto it = w.done.find(ticket);
  if (it == w.done.end() && !w.pending.count(ticket)) return CE_ERR_INVALID_ARG;  // unknown or waited
  // done, or taken meanwhile by another waiter of the same ticket
  w.cv_done.wait(lk, [&] { return (it = w.done.find(ticket)) != w.done.end() || !w.pending.count(ticket); });
  if (it == w.done.end()) return CE_ERR_INVALID_ARG;
  std::snprintf(name_out, 64, "%s", it->second.c_str());
  w.done.erase(it);
  return CE_OK;
}

// ---- VersionBytesBuf (version_bytes.rs:245-309) ----
void ce_vbuf_init(ce_vbuf* b, const uint8_t version[16], const uint8_t* content, size_t len) {
  b->pos = 0;
  std::memcpy(b->version, version, 16);
  b->content = content;
  b->content_len = len;
}

size_t ce_vbuf_remaining(const ce_vbuf* b) { return 16 + b->content_len - b->pos; }

size_t ce_vbuf_chunk(const ce_vbuf* b, const uint8_t** chunk) {
  if (b->pos < 16) {
    *chunk = b->version + b->pos;
    return 16 - b->pos;
  }
  const size_t p = b->pos - 16;
  if (b->content_len <= p) {
    *chunk = b->content;
    return 0;
  }
  *chunk = b->content + p;
  return b->content_len - p;
}

int ce_vbuf_advance(ce_vbuf* b, size_t cnt) {
  if (cnt > ce_vbuf_remaining(b)) return -1;  // the reference asserts (panics)
  b->pos += cnt;
  return 0;
}

size_t ce_vbuf_chunks_vectored(const ce_vbuf* b, const uint8_t** dst_ptr, size_t* dst_len,
                               size_t n_dst) {
  if (n_dst == 0) return 0;
  if (b->pos < 16) {
    dst_ptr[0] = b->version + b->pos;
    dst_len[0] = 16 - b->pos;
    if (n_dst == 1) return 1;
    dst_ptr[1] = b->content;
    dst_len[1] = b->content_len;
    return 2;
  }
  const size_t p = b->pos - 16;
  if (b->content_len == p) return 0;
  dst_ptr[0] = b->content + p;
  dst_len[0] = b->content_len - p;
  return 1;
}

}  // extern "C"
