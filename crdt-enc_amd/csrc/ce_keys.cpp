// ce_keys.cpp -- the key path in front of the hot path: remote meta files -> the key cryptor's
// register -> Keys { latest_key_id: MVReg<Uuid, Uuid>, keys: Orswot<Key, Uuid> } ->
// Keys::latest_key (crdt-enc/src/key_cryptor.rs:35-70), and the key set the core opens with.
//
//   RemoteMeta { storage, cryptor, key_cryptor: MVReg<VersionBytes, Uuid> }   (lib.rs:752-764)
//     stored as VersionBytes(CURRENT_VERSION, to_vec_named(RemoteMeta))      (lib.rs:647-664)
//     read + merged by Core::read_remote_meta_                               (lib.rs:553-612)
//   key_cryptor values: VersionBytes(gpgme CURRENT_VERSION, to_vec_named(Keys)), not encrypted
//     (the gpgme KeyHandler's encryption is a TODO pass-through, crdt-enc-gpgme/src/lib.rs:
//     79-105, 107-129); decode_version_bytes_mvreg_custom_phf merges every value's Keys
//     (crdt-enc/src/utils/mod.rs:94-126).
//
// crdts 7 semantics restated here (host, a handful of keys): VClock, MVReg::merge / read,
// Orswot::merge / apply_rm / apply_deferred / read -- the same statements oracle/crdts.py
// restates for the dot-set fold (parity unpinned).
#include <algorithm>
#include <map>
#include <set>

#include "ce_core.h"

using namespace ce;

namespace {

const uint8_t kGpgmeVersion[16] = {0xe6, 0x9c, 0xb6, 0x8e, 0x7f, 0xbb, 0x41, 0xaa,
                                   0x8d, 0x22, 0x87, 0xea, 0xce, 0x7a, 0x04, 0xc9};

// ---- VClock<Uuid> as a sorted Dots vector (zero counters never stored) ----
Dots vc_norm(Dots d) {
  std::sort(d.begin(), d.end());
  Dots o;
  for (auto& x : d) {
    if (!o.empty() && o.back().first == x.first) o.back().second = x.second;  // BTreeMap: last wins
    else o.push_back(x);
  }
  o.erase(std::remove_if(o.begin(), o.end(), [](const std::pair<Uuid, uint64_t>& x) { return x.second == 0; }),
          o.end());
  return o;
}
uint64_t vc_get(const Dots& v, const Uuid& a) {
  auto it = std::lower_bound(v.begin(), v.end(), a,
                             [](const std::pair<Uuid, uint64_t>& x, const Uuid& k) { return x.first < k; });
  return it != v.end() && it->first == a ? it->second : 0;
}
void vc_apply(Dots& v, const Uuid& a, uint64_t c) {
  auto it = std::lower_bound(v.begin(), v.end(), a,
                             [](const std::pair<Uuid, uint64_t>& x, const Uuid& k) { return x.first < k; });
  if (it != v.end() && it->first == a) {
    if (it->second < c) it->second = c;
  } else if (c) {
    v.insert(it, {a, c});
  }
}
void vc_merge(Dots& v, const Dots& o) {
  for (auto& x : o) vc_apply(v, x.first, x.second);
}
bool vc_le(const Dots& a, const Dots& b) {  // every dot of a covered by b
  for (auto& x : a)
    if (vc_get(b, x.first) < x.second) return false;
  return true;
}
bool vc_lt(const Dots& a, const Dots& b) { return a != b && vc_le(a, b); }
void vc_reset_remove(Dots& v, const Dots& o) {  // drop actors whose counter is <= other's
  Dots r;
  for (auto& x : v)
    if (x.second > vc_get(o, x.first)) r.push_back(x);
  v.swap(r);
}
Dots vc_intersection(const Dots& a, const Dots& b) {
  Dots r;
  for (auto& x : a)
    if (vc_get(b, x.first) == x.second) r.push_back(x);
  return r;
}

struct KeyVal {
  Uuid version{};
  std::vector<uint8_t> bytes;
};

// Key { id: Uuid, key: VersionBytes } -- Eq/Hash/Ord by id only (key_cryptor.rs:109-139)
bool read_version_bytes(Rd& r, KeyVal* out) {
  uint64_t cnt, off;
  if (r.i >= r.n || !is_array_marker(r.p[r.i]) || !rd_array_hdr(r, &cnt) || cnt != 2) return false;
  if (!rd_uuid(r, &off)) return false;
  std::memcpy(out->version.data(), r.p + off, 16);
  return bytes_any(r, &out->bytes);
}
bool read_key(Rd& r, Uuid* id, KeyVal* kv) {
  bool has_id = false, has_key = false;
  return read_struct(r, {"id", "key"}, [&](int f, Rd& q) {
           if (f == 0) {
             uint64_t off;
             if (!rd_uuid(q, &off)) return false;
             std::memcpy(id->data(), q.p + off, 16);
             has_id = true;
             return true;
           }
           has_key = true;
           return read_version_bytes(q, kv);
         }) && has_id && has_key;
}

template <typename V>
struct MVRegT {  // crdts 7 MVReg: vals in Vec order
  std::vector<std::pair<Dots, V>> vals;
  void merge(const MVRegT& o) {
    std::vector<std::pair<Dots, V>> kept;
    for (auto& x : vals) {
      bool dominated = false;
      for (auto& y : o.vals) dominated |= vc_lt(x.first, y.first);
      if (!dominated) kept.push_back(x);
    }
    std::vector<std::pair<Dots, V>> add;
    for (auto& y : o.vals) {
      bool dominated = false, dup = false;
      for (auto& x : kept) {
        dominated |= vc_lt(y.first, x.first);
        dup |= y.first == x.first;
      }
      if (!dominated && !dup) add.push_back(y);
    }
    kept.insert(kept.end(), add.begin(), add.end());
    vals.swap(kept);
  }
};

template <typename V, typename ReadV>
bool read_mvreg(Rd& r, MVRegT<V>* out, ReadV read_v) {
  return read_struct(r, {"vals"}, [&](int, Rd& q) {
    uint64_t cnt;
    if (!rd_array_hdr(q, &cnt) || cnt > q.n - q.i) return false;
    for (uint64_t k = 0; k < cnt; k++) {
      uint64_t two;
      if (q.i >= q.n || !is_array_marker(q.p[q.i]) || !rd_array_hdr(q, &two) || two != 2) return false;
      Dots clock;
      V v;
      if (!read_vclock(q, &clock) || !read_v(q, &v)) return false;
      out->vals.push_back({vc_norm(clock), v});
    }
    return true;
  });
}

struct OrswotKeys {  // crdts 7 Orswot<Key, Uuid>, members identified by Key::id
  Dots clock;
  std::map<Uuid, std::pair<KeyVal, Dots>> entries;
  std::vector<std::pair<Dots, std::set<Uuid>>> deferred;

  void apply_rm(const std::set<Uuid>& members, const Dots& rm) {
    for (auto& m : members) {
      auto it = entries.find(m);
      if (it == entries.end()) continue;
      vc_reset_remove(it->second.second, rm);
      if (it->second.second.empty()) entries.erase(it);
    }
    if (!vc_le(rm, clock)) {
      for (auto& d : deferred)
        if (d.first == rm) {
          d.second.insert(members.begin(), members.end());
          return;
        }
      deferred.push_back({rm, members});
    }
  }
  void apply_deferred() {
    auto d = std::move(deferred);
    deferred.clear();
    for (auto& x : d) apply_rm(x.second, x.first);
  }
  void merge(const OrswotKeys& o) {
    std::map<Uuid, std::pair<KeyVal, Dots>> kept;
    for (auto& e : entries) {
      if (!o.entries.count(e.first)) {
        if (vc_le(e.second.second, o.clock)) continue;  // other has seen it and dropped it
        auto c = e.second;
        vc_reset_remove(c.second, o.clock);
        kept[e.first] = c;
      } else {
        kept[e.first] = e.second;
      }
    }
    entries.swap(kept);
    for (auto& e : o.entries) {
      auto it = entries.find(e.first);
      if (it != entries.end()) {
        Dots common = vc_intersection(e.second.second, it->second.second);
        Dots a = e.second.second, b = it->second.second;
        vc_reset_remove(a, clock);
        vc_reset_remove(b, o.clock);
        vc_merge(common, a);
        vc_merge(common, b);
        if (common.empty()) entries.erase(it);
        else it->second = {e.second.first, common};  // the other side's Key (HashMap insert)
      } else {
        if (vc_le(e.second.second, clock)) continue;  // seen and dropped
        auto c = e.second;
        vc_reset_remove(c.second, clock);
        entries[e.first] = c;
      }
    }
    for (auto& d : o.deferred) apply_rm(d.second, d.first);
    vc_merge(clock, o.clock);
    apply_deferred();
  }
};

bool read_orswot_keys(Rd& r, OrswotKeys* o) {
  return read_struct(r, {"clock", "entries", "deferred"}, [&](int f, Rd& q) {
    if (f == 0) {
      Dots c;
      if (!read_vclock(q, &c)) return false;
      o->clock = vc_norm(c);
      return true;
    }
    uint64_t cnt;
    if (!rd_map_hdr(q, &cnt) || cnt > q.n - q.i) return false;
    for (uint64_t k = 0; k < cnt; k++) {
      if (f == 1) {
        Uuid id;
        KeyVal kv;
        Dots c;
        if (!read_key(q, &id, &kv) || !read_vclock(q, &c)) return false;
        o->entries[id] = {kv, vc_norm(c)};  // HashMap: a repeated key overwrites
      } else {
        Dots c;
        uint64_t nm;
        if (!read_vclock(q, &c) || !rd_array_hdr(q, &nm) || nm > q.n - q.i) return false;
        std::set<Uuid> ms;
        for (uint64_t j = 0; j < nm; j++) {
          Uuid id;
          KeyVal kv;
          if (!read_key(q, &id, &kv)) return false;
          ms.insert(id);
        }
        o->deferred.push_back({vc_norm(c), ms});
      }
    }
    return true;
  });
}

bool read_uuid_v(Rd& r, Uuid* u) {
  uint64_t off;
  if (!rd_uuid(r, &off)) return false;
  std::memcpy(u->data(), r.p + off, 16);
  return true;
}

}  // namespace

struct ce_keys {
  MVRegT<Uuid> latest;
  OrswotKeys keys;
  void merge(const ce_keys& o) {  // Keys::merge (key_cryptor.rs:42-50)
    latest.merge(o.latest);
    keys.merge(o.keys);
  }
};

namespace {

bool decode_keys(const uint8_t* p, size_t n, ce_keys* k) {
  Rd r{p, n, 0};
  return read_struct(r, {"latest_key_id", "keys"}, [&](int f, Rd& q) {
    if (f == 0) return read_mvreg<Uuid>(q, &k->latest, read_uuid_v);
    return read_orswot_keys(q, &k->keys);
  });
}

int put_key(const std::pair<KeyVal, Dots>& e, uint8_t ver[16], uint8_t* key, size_t cap, size_t* len) {
  if (len) *len = e.first.bytes.size();
  if (ver) std::memcpy(ver, e.first.version.data(), 16);
  if (key) {
    if (cap < e.first.bytes.size()) return CE_ERR_INVALID_ARG;
    std::memcpy(key, e.first.bytes.data(), e.first.bytes.size());
  }
  return CE_OK;
}

}  // namespace

extern "C" {

int ce_keys_decode(const uint8_t* msgpack, size_t len, ce_keys** out) {
  if (!out || (len && !msgpack)) return CE_ERR_INVALID_ARG;
  auto* k = new ce_keys();
  if (!decode_keys(msgpack, len, k)) {
    delete k;
    return CE_ERR_DECODE;
  }
  *out = k;
  return CE_OK;
}

int ce_keys_from_remote_metas(const uint8_t* blob, const uint64_t* offs, uint32_t n, ce_keys** out) {
  if (!out || (n && (!blob || !offs))) return CE_ERR_INVALID_ARG;
  // RemoteMeta.key_cryptor of every file, merged (lib.rs:585-593: remote_meta.merge(meta))
  MVRegT<KeyVal> reg;
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* f = blob + offs[i];
    const size_t fl = offs[i + 1] - offs[i];
    if (fl < 16) return CE_ERR_OUTER_LEN;                                 // VersionBytes::deserialize
    if (std::memcmp(f, kCoreVersion, 16) != 0) return CE_ERR_OUTER_VERSION;  // lib.rs:578
    Rd r{f + 16, fl - 16, 0};
    MVRegT<KeyVal> kc;
    const bool ok = read_struct(r, {"storage", "cryptor", "key_cryptor"}, [&](int fi, Rd& q) {
      if (fi != 2) return skip_any(q);
      return read_mvreg<KeyVal>(q, &kc, read_version_bytes);
    });
    if (!ok) return CE_ERR_DECODE;
    reg.merge(kc);
  }
  // KeyHandler::set_remote_meta -> decode_version_bytes_mvreg_custom_phf (utils/mod.rs:94-126):
  // every value's version checked against the gpgme SUPPORTED_VERSIONS, Keys merged
  auto* k = new ce_keys();
  for (auto& v : reg.vals) {
    if (std::memcmp(v.second.version.data(), kGpgmeVersion, 16) != 0) {
      delete k;
      return CE_ERR_PT_VERSION;
    }
    ce_keys one;
    if (!decode_keys(v.second.bytes.data(), v.second.bytes.size(), &one)) {
      delete k;
      return CE_ERR_DECODE;
    }
    k->merge(one);
  }
  *out = k;
  return CE_OK;
}

int ce_keys_merge(ce_keys* k, const ce_keys* other) {
  if (!k || !other) return CE_ERR_INVALID_ARG;
  k->merge(*other);
  return CE_OK;
}

void ce_keys_free(ce_keys* k) { delete k; }

uint32_t ce_keys_count(const ce_keys* k) { return k ? (uint32_t)k->keys.entries.size() : 0; }

int ce_keys_latest(const ce_keys* k, uint8_t id_out[16], uint8_t key_version_out[16], uint8_t* key_out,
                   size_t cap, size_t* key_len) {
  if (!k) return CE_ERR_INVALID_ARG;
  // latest_key_id.read().val mapped to keys.read().val, min by id (key_cryptor.rs:59-70)
  const Uuid* best = nullptr;
  std::vector<const Uuid*> taken;
  for (auto& v : k->latest.vals) {
    // keys.take(&id) removes the key it returns, so a repeated id finds none: the reference
    // panics (:67) on a missing key and on a repeat alike
    if (!k->keys.entries.count(v.second)) return CE_ERR_DECODE;
    for (const Uuid* t : taken)
      if (*t == v.second) return CE_ERR_DECODE;
    taken.push_back(&v.second);
    if (!best || v.second < *best) best = &v.second;
  }
  if (!best) return CE_ERR_NO_KEY;
  if (id_out) std::memcpy(id_out, best->data(), 16);
  return put_key(k->keys.entries.at(*best), key_version_out, key_out, cap, key_len);
}

int ce_keys_get(const ce_keys* k, const uint8_t id[16], uint8_t key_version_out[16], uint8_t* key_out,
                size_t cap, size_t* key_len) {
  if (!k || !id) return CE_ERR_INVALID_ARG;
  Uuid u;
  std::memcpy(u.data(), id, 16);
  auto it = k->keys.entries.find(u);
  if (it == k->keys.entries.end()) return CE_ERR_NO_KEY;  // Keys::get_key -> None (:55-57)
  return put_key(it->second, key_version_out, key_out, cap, key_len);
}

int ce_keys_at(const ce_keys* k, uint32_t i, uint8_t id_out[16], uint8_t key_version_out[16],
               uint8_t* key_out, size_t cap, size_t* key_len) {
  if (!k || i >= k->keys.entries.size()) return CE_ERR_INVALID_ARG;
  auto it = k->keys.entries.begin();
  std::advance(it, i);
  if (id_out) std::memcpy(id_out, it->first.data(), 16);
  return put_key(it->second, key_version_out, key_out, cap, key_len);
}

int ce_core_set_keys(ce_core* c, const ce_keys* k) {
  if (!c || !k) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  uint8_t id[16], ver[16];
  size_t len = 0;
  int rc = ce_keys_latest(k, id, ver, nullptr, 0, &len);
  if (rc) return c->ctx->fail(rc, rc == CE_ERR_NO_KEY ? "no latest key" : "latest key id without a key");
  std::vector<uint8_t> key(len);
  ce_keys_latest(k, id, ver, key.data(), len, &len);
  std::memcpy(c->key_version, ver, 16);
  c->key = key;
  c->has_key = true;
  // the other keys, in id order: tried on authentication failures with CE_OPEN_MULTI_KEY
  c->alt_keys.clear();
  for (auto& e : k->keys.entries) {
    if (std::memcmp(e.first.data(), id, 16) == 0) continue;
    AltKey a;
    std::memcpy(a.version, e.second.first.version.data(), 16);
    a.key = e.second.first.bytes;
    c->alt_keys.push_back(a);
  }
  return CE_OK;
}

}  // extern "C"
