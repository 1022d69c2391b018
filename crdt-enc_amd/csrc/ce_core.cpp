// ce_core.cpp -- Core<S, Storage, Cryptor, _> (crdt-enc/src/lib.rs:188-723), driving the GPU
// batch engine.  S = VClock<Uuid> / GCounter<Uuid> live here; S = Orswot<u64, Uuid> /
// MVReg<u64, Uuid> (the dot-set kinds) dispatch to ce_dotset_host.cpp.
//
// State layout: a host-built open-addressing actor table (UUID -> dense slot) mirrored in HBM;
// the CRDT state (VClock dots / GCounter.inner) is a dense u64[cap] max-register array in HBM;
// next_op_versions (lib.rs:741) is a dense u64[cap] on the host (the version gate runs there
// while the GPU decrypts).  Serialization sorts slots by UUID bytes = BTreeMap order.
#include <algorithm>
#include <atomic>
#include <cstdio>
#include <functional>
#include <set>

#include "ce_core.h"
#include "ce_shard.h"

using namespace ce;

namespace ce {

// ---------------------------------------------------------------------------------------
// msgpack writer (rmp-serde to_vec_named)
// ---------------------------------------------------------------------------------------

// ---------------------------------------------------------------------------------------
// host-side msgpack reading (states, local ops, local meta, exotic envelopes)
// ---------------------------------------------------------------------------------------
// skip one value, recursion depth bounded like rmp-serde's default (1024)
bool skip_any(Rd& r, int depth) {
  if (depth > 1024) return false;
  uint64_t at, cnt = 0;
  if (r.i >= r.n) return false;
  const uint8_t m = r.p[r.i];
  bool cont = false;
  if ((m & 0xf0) == 0x80) { r.i++; cnt = 2ull * (m & 15); cont = true; }
  else if ((m & 0xf0) == 0x90) { r.i++; cnt = m & 15; cont = true; }
  else if (m == 0xdc || m == 0xdd || m == 0xde || m == 0xdf) {
    r.i++;
    if (!rd_be(r, (m == 0xdc || m == 0xde) ? 2 : 4, &cnt)) return false;
    if (m >= 0xde) cnt *= 2;
    cont = true;
  }
  if (cont) {
    for (uint64_t k = 0; k < cnt; k++)
      if (!skip_any(r, depth + 1)) return false;
    return true;
  }
  Rd q = r;
  int s = rd_skip(q);  // scalar / bin / str / ext: no recursion needed
  if (s != 1) return false;
  r = q;
  (void)at;
  return true;
}

// serde_bytes Cow<[u8]> in any accepted form (bin, str, array of u8)
bool bytes_any(Rd& r, std::vector<uint8_t>* out) {
  if (r.i >= r.n) return false;
  if (is_array_marker(r.p[r.i])) {
    uint64_t cnt, v;
    if (!rd_array_hdr(r, &cnt) || cnt > r.n) return false;
    out->clear();
    for (uint64_t k = 0; k < cnt; k++) {
      if (!rd_u64(r, &v) || v > 255) return false;
      out->push_back((uint8_t)v);
    }
    return true;
  }
  int kind;
  uint64_t off, len;
  if (!rd_binstr(r, &kind, &off, &len)) return false;
  out->assign(r.p + off, r.p + off + len);
  return true;
}

// derive(Deserialize) struct: map (any key order; unknown ignored; duplicates rejected) or
// array of exactly nf.  cb(field, rd) reads a value.
bool read_struct(Rd& r, const std::vector<const char*>& names,
                 const std::function<bool(int, Rd&)>& cb) {
  const int nf = (int)names.size();
  if (r.i >= r.n) return false;
  uint64_t cnt;
  if (is_array_marker(r.p[r.i])) {
    if (!rd_array_hdr(r, &cnt) || cnt != (uint64_t)nf) return false;
    for (int f = 0; f < nf; f++)
      if (!cb(f, r)) return false;
    return true;
  }
  if (!rd_map_hdr(r, &cnt)) return false;
  unsigned seen = 0;
  for (uint64_t k = 0; k < cnt; k++) {
    int f;
    const uint8_t m = r.i < r.n ? r.p[r.i] : 0xc1;
    if (is_binstr_marker(m)) {
      int kind;
      uint64_t off, l;
      if (!rd_binstr(r, &kind, &off, &l)) return false;
      f = nf;
      for (int j = 0; j < nf; j++)
        if (std::strlen(names[j]) == l && std::memcmp(names[j], r.p + off, l) == 0) f = j;
    } else {
      uint64_t v;
      if (!rd_u64(r, &v)) return false;
      f = v < (uint64_t)nf ? (int)v : nf;
    }
    if (f == nf) {
      if (!skip_any(r)) return false;
      continue;
    }
    if (seen & (1u << f)) return false;
    seen |= 1u << f;
    if (!cb(f, r)) return false;
  }
  return seen == (1u << nf) - 1;
}

// VClock { dots: BTreeMap<Uuid, u64> }: later duplicate keys overwrite earlier ones
bool read_vclock(Rd& r, Dots* out) {
  // dots map: a later duplicate key overwrites the earlier value (BTreeMap::insert).  Keys in
  // strictly ascending order (what to_vec_named writes) cannot repeat: no lookup structure.
  auto dots = [&](Rd& q) {
    uint64_t cnt;
    if (!rd_map_hdr(q, &cnt) || cnt > q.n - q.i) return false;
    const size_t base = out->size();
    bool ascending = true;
    for (uint64_t k = 0; k < cnt; k++) {
      uint64_t off, c;
      if (!rd_uuid(q, &off) || !rd_u64(q, &c)) return false;
      Uuid u;
      std::memcpy(u.data(), q.p + off, 16);
      if (k && !(out->back().first < u)) ascending = false;
      out->push_back({u, c});
    }
    if (!ascending) {
      Dots v(out->begin() + base, out->end());
      out->resize(base);
      std::unordered_map<Uuid, size_t, UuidHash> idx;
      for (auto& d : v) {
        auto it = idx.find(d.first);
        if (it != idx.end()) (*out)[it->second].second = d.second;
        else { idx[d.first] = out->size(); out->push_back(d); }
      }
    }
    return true;
  };
  // canonical struct form: fixmap(1) "dots"
  if (r.n - r.i >= 6 && r.p[r.i] == 0x81 && r.p[r.i + 1] == 0xa4 && std::memcmp(r.p + r.i + 2, "dots", 4) == 0) {
    r.i += 6;
    return dots(r);
  }
  return read_struct(r, {"dots"}, [&](int, Rd& q) { return dots(q); });
}

// StateWrapper<S> { next_op_versions: VClock, state: S } (lib.rs:739-743)
bool read_state_wrapper(const uint8_t* p, size_t n, int kind, Dots* nov, Dots* st) {
  Rd r{p, n, 0};
  return read_struct(r, {"next_op_versions", "state"}, [&](int f, Rd& q) {
    if (f == 0) return read_vclock(q, nov);
    if (kind == CE_STATE_GCOUNTER)
      return read_struct(q, {"inner"}, [&](int, Rd& q2) { return read_vclock(q2, st); });
    return read_vclock(q, st);
  });
}

// Vec<Dot<Uuid>> (lib.rs:507)
bool read_dots(const uint8_t* p, size_t n, Dots* out) {
  Rd r{p, n, 0};
  uint64_t cnt;
  if (!rd_array_hdr(r, &cnt) || cnt > n) return false;
  for (uint64_t k = 0; k < cnt; k++) {
    uint64_t aoff = 0, c = 0;
    Rd q = r;
    int ok = parse_dot(q, &aoff, &c);
    if (ok < 0) {
      // too deep for the shared parser's bounded stack: host recursion
      bool has_a = false, has_c = false;
      Uuid a{};
      if (!read_struct(r, {"actor", "counter"}, [&](int f, Rd& s) {
            if (f == 0) {
              uint64_t o;
              if (!rd_uuid(s, &o)) return false;
              std::memcpy(a.data(), s.p + o, 16);
              has_a = true;
              return true;
            }
            has_c = true;
            return rd_u64(s, &c);
          }) || !has_a || !has_c)
        return false;
      out->push_back({a, c});
      continue;
    }
    if (ok == 0) return false;
    Uuid a;
    std::memcpy(a.data(), q.p + aoff, 16);
    out->push_back({a, c});
    r = q;
  }
  return true;
}

// Cryptor envelope in any accepted encoding -> canonical bytes (device decodes only the
// in-place forms; an array-of-u8 byte string or deep nesting comes here).
int32_t normalize_envelope(const uint8_t* enc, size_t len, std::vector<uint8_t>* canon) {
  Rd r{enc, len, 0};
  uint64_t cnt;
  if (r.n == 0 || !is_array_marker(r.p[0]) || !rd_array_hdr(r, &cnt) || cnt != 2)
    return CE_ERR_PARSE_VBOX;
  uint64_t voff;
  std::vector<uint8_t> box;
  if (!rd_uuid(r, &voff) || !bytes_any(r, &box)) return CE_ERR_PARSE_VBOX;
  if (std::memcmp(enc + voff, kBoxVersion, 16) != 0) return CE_ERR_DATA_VERSION;
  std::vector<uint8_t> nonce, ed;
  Rd q{box.data(), box.size(), 0};
  if (!read_struct(q, {"nonce", "enc_data"},
                   [&](int f, Rd& s) { return bytes_any(s, f == 0 ? &nonce : &ed); }))
    return CE_ERR_PARSE_ENCBOX;
  if (nonce.size() != 24) return CE_ERR_NONCE_LEN;
  if (ed.size() < 16) return CE_ERR_AUTH;
  canon->resize(128);
  const uint64_t h = put_envelope_header(canon->data(), ed.size() - 16, nonce.data());
  canon->resize(h);
  canon->insert(canon->end(), ed.begin(), ed.end());
  return CE_OK;
}

// ---------------------------------------------------------------------------------------
// actor table
// ---------------------------------------------------------------------------------------
// The actor table is kept at most 1/4 full: linear probing then averages ~1.17 probes per
// successful lookup (1.5 at 1/2), and every probe of a device lookup is a dependent L2 load --
// C2 variant B resolves one per Dot.
static constexpr uint64_t kTableLoadInv = 4;

uint32_t probe_slot(const std::vector<ActorSlot>& t, uint32_t mask, const Uuid& u, bool* found) {
  uint32_t w[4];
  std::memcpy(w, u.data(), 16);
  uint32_t h = actor_hash(w[0], w[1], w[2], w[3]) & mask;
  for (;;) {
    if (!t[h].used) { *found = false; return h; }
    if (std::memcmp(t[h].k, w, 16) == 0) { *found = true; return h; }
    h = (h + 1) & mask;
  }
}

// DecodeArgs.nil_actor: whether the device lookups must take the two-load probe (the nil UUID
// is the one used key that reads like an empty slot, ce_device.h lookup_slot1)
static int table_has_nil(ce_core* c) {
  bool found = false;
  (void)probe_slot(c->h_table, c->cap - 1, Uuid{}, &found);
  return found ? 1 : 0;
}

int table_init(ce_core* c, uint32_t cap) {
  c->table_gen++;
  c->cap = cap;
  c->size = 0;
  c->h_table.assign(cap, ActorSlot{});
  c->slot_actor.assign(cap, Uuid{});
  c->id_actor.clear();
  c->nov.assign(cap, 0);
  c->slot_of.clear();
  c->table_dirty = true;
  hipError_t e;
  if ((e = c->d_table.reserve(cap * sizeof(ActorSlot))) || (e = c->d_state.reserve(cap * 8ull)) ||
      (e = c->d_batch.reserve(cap * 8ull)) || (e = c->d_tmp.reserve(cap * 8ull)))
    return c->ctx->hip_fail(e, "actor table");
  if ((e = hipMemsetAsync(c->d_state.p, 0, cap * 8ull, c->ctx->stream)))
    return c->ctx->hip_fail(e, "actor table");
  return CE_OK;
}

int table_upload(ce_core* c) {
  if (!c->table_dirty) return CE_OK;
  hipError_t e = hipMemcpyAsync(c->d_table.p, c->h_table.data(), c->cap * sizeof(ActorSlot),
                                hipMemcpyHostToDevice, c->ctx->stream);
  if (e) return c->ctx->hip_fail(e, "table upload");
  // the host vector may be rewritten before the copy runs: wait (table changes are rare)
  if ((e = stream_wait(c->ctx->stream))) return c->ctx->hip_fail(e, "table upload");
  c->table_dirty = false;
  return CE_OK;
}

int table_grow(ce_core* c) {
  // rehash into 2x capacity; move the dense state (device) and nov (host) with it
  const uint32_t old_cap = c->cap;
  std::vector<uint64_t> st(old_cap);
  hipError_t e;
  if ((e = hipMemcpyAsync(st.data(), c->d_state.p, old_cap * 8ull, hipMemcpyDeviceToHost,
                          c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "grow");
  std::vector<Uuid> actors;
  std::vector<uint64_t> nov, sv;
  std::vector<uint32_t> ids;
  for (uint32_t s = 0; s < old_cap; s++)
    if (c->h_table[s].used) {
      actors.push_back(c->slot_actor[s]);
      nov.push_back(c->nov[s]);
      sv.push_back(st[s]);
      ids.push_back(c->h_table[s].pad[0]);
    }
  const std::vector<Uuid> id_actor = c->id_actor;
  // keep insertion order stable: re-insert in the old slot order
  const uint32_t reg = c->registered;
  DevBuf keep_state;
  int rc = table_init(c, old_cap * 2);
  if (rc) return rc;
  std::vector<uint64_t> nst(c->cap, 0);
  for (size_t i = 0; i < actors.size(); i++) {
    bool found;
    const uint32_t s = probe_slot(c->h_table, c->cap - 1, actors[i], &found);
    std::memcpy(c->h_table[s].k, actors[i].data(), 16);
    c->h_table[s].used = 1;
    c->h_table[s].pad[0] = ids[i];
    c->slot_actor[s] = actors[i];
    c->slot_of[actors[i]] = s;
    c->nov[s] = nov[i];
    nst[s] = sv[i];
    c->size++;
  }
  c->id_actor = id_actor;
  c->registered = reg;
  if ((e = hipMemcpyAsync(c->d_state.p, nst.data(), c->cap * 8ull, hipMemcpyHostToDevice,
                          c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "grow");
  return CE_OK;
}

int insert_actor(ce_core* c, const Uuid& u, uint32_t* slot) {
  auto it = c->slot_of.find(u);
  if (it != c->slot_of.end()) { *slot = it->second; return CE_OK; }
  if ((c->size + 1) * kTableLoadInv > c->cap) {
    int rc = table_grow(c);
    if (rc) return rc;
  }
  bool found;
  const uint32_t s = probe_slot(c->h_table, c->cap - 1, u, &found);
  std::memcpy(c->h_table[s].k, u.data(), 16);
  c->h_table[s].used = 1;
  c->h_table[s].pad[0] = (uint32_t)c->id_actor.size();
  c->id_actor.push_back(u);
  c->slot_actor[s] = u;
  c->slot_of[u] = s;
  c->size++;
  c->table_dirty = true;
  c->table_gen++;
  *slot = s;
  return CE_OK;
}

int download_state(ce_core* c, std::vector<uint64_t>* st) {
  st->resize(c->cap);
  hipError_t e;
  if ((e = hipMemcpyAsync(st->data(), c->d_state.p, c->cap * 8ull, hipMemcpyDeviceToHost,
                          c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "state download");
  return CE_OK;
}

// max-merge host dots into the device state (VClock::merge / apply)
// slots of m actors (16 bytes each) after a table growth moved the ones handed out before it
void refresh_slots(ce_core* c, const uint8_t* actors, uint32_t m, std::vector<uint32_t>* slots) {
  for (uint32_t a = 0; a < m; a++) {
    Uuid u;
    std::memcpy(u.data(), actors + 16ull * a, 16);
    (*slots)[a] = c->slot_of.at(u);
  }
}

int merge_dots_host(ce_core* c, const Dots& dots) {
  if (dots.empty()) return CE_OK;
  std::vector<std::pair<uint32_t, uint64_t>> sv;
  const uint64_t gen0 = c->table_gen;
  for (auto& d : dots) {
    uint32_t s;
    int rc = insert_actor(c, d.first, &s);
    if (rc) return rc;
    sv.push_back({s, d.second});
  }
  // a growth during the loop moved every slot handed out before it
  if (c->table_gen != gen0)
    for (size_t i = 0; i < dots.size(); i++) sv[i].first = c->slot_of.at(dots[i].first);
  std::vector<uint64_t> dense(c->cap, 0);
  for (auto& p : sv) dense[p.first] = std::max(dense[p.first], p.second);
  hipError_t e;
  if ((e = hipMemcpyAsync(c->d_tmp.p, dense.data(), c->cap * 8ull, hipMemcpyHostToDevice,
                          c->ctx->stream)) ||
      (e = launch_merge_max(c->ctx->stream, c->d_state.as<unsigned long long>(),
                            c->d_tmp.as<unsigned long long>(), c->cap)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "merge dots");
  return CE_OK;
}

// used slots in UUID byte order (BTreeMap iteration order), cached per table generation
void ensure_sorted(ce_core* c) {
  if (c->sorted_gen == c->table_gen) return;
  c->sorted_slots.clear();
  for (uint32_t s = 0; s < c->cap; s++)
    if (c->h_table[s].used) c->sorted_slots.push_back(s);
  std::sort(c->sorted_slots.begin(), c->sorted_slots.end(), [&](uint32_t a, uint32_t b) {
    return std::memcmp(c->slot_actor[a].data(), c->slot_actor[b].data(), 16) < 0;
  });
  c->sorted_gen = c->table_gen;
}

int serialize_state(ce_core* c, std::vector<uint8_t>* out) {
  if (is_dotset_kind(c->kind)) return ds_serialize(c, out);
  std::vector<uint64_t> st;
  int rc = download_state(c, &st);
  if (rc) return rc;
  ensure_sorted(c);
  const std::vector<uint32_t>& slots = c->sorted_slots;
  size_t n_nov = 0, n_st = 0;
  for (uint32_t s : slots) { n_nov += c->nov[s] != 0; n_st += st[s] != 0; }
  Wr w;
  w.b.swap(*out);  // reuse the caller's capacity
  w.b.clear();
  w.b.reserve(64 + 28 * (n_nov + n_st));
  w.map(2);
  w.str("next_op_versions");
  w.map(1);
  w.str("dots");
  w.map(n_nov);
  for (uint32_t s : slots)
    if (c->nov[s]) { w.bin(c->slot_actor[s].data(), 16); w.uint(c->nov[s]); }
  w.str("state");
  if (c->kind == CE_STATE_GCOUNTER) { w.map(1); w.str("inner"); }
  w.map(1);
  w.str("dots");
  w.map(n_st);
  for (uint32_t s : slots)
    if (st[s]) { w.bin(c->slot_actor[s].data(), 16); w.uint(st[s]); }
  out->swap(w.b);
  return CE_OK;
}

KeyRef key_of(ce_core* c) { return KeyRef{c->key_version, c->key.data(), c->key.size()}; }

ce_ctx* aux_ctx(ce_core* c) {
  if (!c->aux) {
    c->aux = new ce_ctx();
    c->aux->device = c->ctx->device;
    c->aux->own_stream = false;
  }
  c->aux->stream = c->ctx->stream;  // follows ce_ctx_set_stream
  return c->aux;
}

// Open one file (host bytes) with the aux context: returns status, plaintext.
int open_one(ce_core* c, const uint8_t* file, size_t flen, bool outer, int32_t* st,
             std::vector<uint8_t>* pt) {
  ce_ctx* a = aux_ctx(c);
  const uint64_t offs[2] = {0, flen};
  hipError_t e;
  if ((e = a->blob.reserve(flen + 64)) || (e = a->offs.reserve(64)) ||
      (e = a->out.reserve(flen + 128)) || (e = a->status.reserve(64)))
    return a->hip_fail(e, "open_one");
  if ((e = hipMemcpyAsync(a->blob.p, file, flen, hipMemcpyHostToDevice, a->stream)) ||
      (e = hipMemcpyAsync(a->offs.p, offs, 16, hipMemcpyHostToDevice, a->stream)))
    return a->hip_fail(e, "open_one");
  int rc = device_open(a, a->blob.as<uint8_t>(), a->offs.as<uint64_t>(), 1, flen, outer, key_of(c),
                       a->out.as<uint8_t>(), a->status.as<int32_t>(), false);
  if (rc) return rc;
  FileParams P;
  if ((e = hipMemcpyAsync(&P, a->params.p, sizeof P, hipMemcpyDeviceToHost, a->stream)) ||
      (e = hipMemcpyAsync(st, a->status.p, 4, hipMemcpyDeviceToHost, a->stream)) ||
      (e = stream_wait(a->stream)))
    return a->hip_fail(e, "open_one");
  if (*st == CE_OK) {
    pt->resize(P.len);
    if (P.len && ((e = hipMemcpyAsync(pt->data(), a->out.as<uint8_t>() + P.out_off, P.len,
                                      hipMemcpyDeviceToHost, a->stream)) ||
                  (e = stream_wait(a->stream))))
      return a->hip_fail(e, "open_one");
  }
  return CE_OK;
}

// Files whose envelope the device left to the host: normalize, open the canonical form on the
// GPU, and patch the batch (plaintext into ctx->out at the file's slot, params.len, status).
int resolve_host_parse(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                       bool outer) {
  ce_ctx* ctx = c->ctx;
  std::vector<int32_t> st(n);
  hipError_t e;
  if ((e = hipMemcpyAsync(st.data(), ctx->status.p, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
      (e = stream_wait(ctx->stream)))
    return ctx->hip_fail(e, "host parse");
  for (uint32_t i = 0; i < n; i++) {
    if (st[i] != kStatusHostParse) continue;
    uint64_t o[2];
    FileParams P;
    if ((e = hipMemcpy(o, d_offs + i, 16, hipMemcpyDeviceToHost)) ||
        (e = hipMemcpy(&P, ctx->params.as<FileParams>() + i, sizeof P, hipMemcpyDeviceToHost)))
      return ctx->hip_fail(e, "host parse");
    std::vector<uint8_t> file(o[1] - o[0]);
    if ((e = hipMemcpy(file.data(), d_blob + o[0], file.size(), hipMemcpyDeviceToHost)))
      return ctx->hip_fail(e, "host parse");
    const size_t pre = outer ? 16 : 0;
    std::vector<uint8_t> canon;
    int32_t s = normalize_envelope(file.data() + pre, file.size() - pre, &canon);
    std::vector<uint8_t> pt;
    if (s == CE_OK) {
      std::vector<uint8_t> nf(file.begin(), file.begin() + pre);
      nf.insert(nf.end(), canon.begin(), canon.end());
      int rc = open_one(c, nf.data(), nf.size(), outer, &s, &pt);
      if (rc) return rc;
    }
    FileParams NP = P;
    NP.status = s;
    NP.len = s == CE_OK ? (uint32_t)pt.size() : 0;
    if ((s == CE_OK && !pt.empty() &&
         (e = hipMemcpy(ctx->out.as<uint8_t>() + P.out_off, pt.data(), pt.size(), hipMemcpyHostToDevice))) ||
        (e = hipMemcpy(ctx->params.as<FileParams>() + i, &NP, sizeof NP, hipMemcpyHostToDevice)) ||
        (e = hipMemcpy(ctx->status.as<int32_t>() + i, &s, 4, hipMemcpyHostToDevice)))
      return ctx->hip_fail(e, "host parse");
  }
  return CE_OK;
}

int ensure_supported(ce_core* c) {
  if (c->supported_on_device) return CE_OK;  // fixed at open (lib.rs:227-228): upload once
  const size_t bytes = c->supported.size() * 16;
  hipError_t e;
  if ((e = c->d_supported.reserve(bytes + 16))) return c->ctx->hip_fail(e, "supported");
  if (bytes && (e = hipMemcpyAsync(c->d_supported.p, c->supported.data(), bytes,
                                   hipMemcpyHostToDevice, c->ctx->stream)))
    return c->ctx->hip_fail(e, "supported");
  if ((e = stream_wait(c->ctx->stream))) return c->ctx->hip_fail(e, "supported");
  c->supported_on_device = true;
  return CE_OK;
}

// Host version gate (lib.rs:519-538) for batches the device gate does not cover (actors split
// into several runs, non-consecutive versions).  Returns the first gap index (n if none).
uint32_t host_gate(const uint32_t* fa, const uint64_t* fv, uint32_t n, std::vector<uint64_t>* expect,
                   uint8_t* apply) {
  uint32_t first_gap = n;
  for (uint32_t i = 0; i < n; i++) {
    const uint32_t a = fa[i];
    const uint64_t v = fv[i];
    if (v < (*expect)[a]) { apply[i] = 0; continue; }   // already read
    if (v > (*expect)[a]) { first_gap = i; break; }     // "Unexpected op version"
    apply[i] = 1;
    (*expect)[a] = v + 1;
  }
  for (uint32_t i = first_gap; i < n; i++) apply[i] = 0;
  return first_gap;
}

// Core::read_remote_ops after Storage::load_ops (lib.rs:495-546), files and per-file metadata
// resident in HBM (d_fa = local actor index per file, d_fv = version per file).
// after_commit (optional): called once the device commit (k_merge_max_if) is enqueued, before
// the host waits -- work it enqueues on the stream overlaps the fused kernel's run on the host
// side.  merged_out: whether the commit happened on the device (the fast path).
using AfterCommit = std::function<int(NovApply&)>;

// ingest_ops_dev_once asks for a fresh pass: actors found while decoding plaintext that is not
// re-opened by the fused kernel (host-parse envelopes, CE_OPEN_MULTI_KEY retries) grew the actor
// table, so every slot moved and the partial batch state is stale.  The new actors stay in the
// table, so the next pass finds them.
static constexpr int kRestartIngest = -1000;

// Decode + fold the files flagged in d_mask (n bytes) whose plaintext sits in ctx->out
// (k_decode_dots), with actor-table misses resolved as the fused path does (insert, upload,
// fold the missed files again).  Returns kRestartIngest when the table had to grow.
int decode_only_resolving(ce_core* c, DecodeArgs& da, uint32_t n, uint8_t* d_mask) {
  ce_ctx* ctx = c->ctx;
  uint32_t* hc = ctx->h_counters.as<uint32_t>();
  hipError_t e;
  for (int round = 0;; round++) {
    da.only = d_mask;
    da.large_only = 0;
    da.table = c->d_table.as<ActorSlot>();
    da.mask = c->cap - 1;
    da.nil_actor = table_has_nil(c);
    da.batch = c->d_batch.as<unsigned long long>();
    if ((e = hipMemsetAsync(ctx->counters.as<uint32_t>() + 4, 0, 4, ctx->stream)) ||
        (e = hipMemsetAsync(ctx->refold.p, 0, n, ctx->stream)) ||
        (e = launch_decode_dots(ctx->stream, da, grid_waves_for(n))) ||
        (e = hipMemcpyAsync(hc, ctx->counters.p, 64, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "decode plaintext");
    if (hc[4] == 0) return CE_OK;
    if (round > 64) return ctx->fail(CE_ERR_DEVICE, "actor table did not converge");
    const uint32_t nm = std::min<uint32_t>(hc[4], 65536);
    std::vector<uint4> ml(nm);
    if ((e = hipMemcpyAsync(ml.data(), ctx->miss.p, nm * 16ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = hipMemcpyAsync(d_mask, ctx->refold.p, n, hipMemcpyDeviceToDevice, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "miss");
    const uint32_t old_cap = c->cap;
    for (auto& x : ml) {
      Uuid u;
      std::memcpy(u.data(), &x, 16);
      uint32_t s;
      int rc = insert_actor(c, u, &s);
      if (rc) return rc;
    }
    int rc = table_upload(c);
    if (rc) return rc;
    if (c->cap != old_cap) return kRestartIngest;
  }
}

// CE_OPEN_MULTI_KEY (beyond the reference): the files that failed authentication
// under the latest key are opened again under each other key of the set, in id order (whole
// batch opened per key with device_open, plaintext into ctx->out; only the files still failing
// and now opening are decoded and folded).  st: per-file statuses, updated in place.
int retry_alt_keys(ce_core* c, DecodeArgs& da, const uint8_t* d_blob, const uint64_t* d_offs,
                   uint32_t n, uint64_t blob_len, std::vector<int32_t>& st) {
  ce_ctx* ctx = c->ctx;
  hipError_t e;
  std::vector<int32_t> sk(n);
  std::vector<uint8_t> sel(n);
  for (const AltKey& ak : c->alt_keys) {
    bool any = false;
    for (uint32_t i = 0; i < n; i++) any |= st[i] == CE_ERR_AUTH;
    if (!any) break;
    const KeyRef kr{ak.version, ak.key.data(), ak.key.size()};
    int rc = device_open(ctx, d_blob, d_offs, n, blob_len, true, kr, ctx->out.as<uint8_t>(),
                         ctx->status.as<int32_t>(), false);
    if (rc) return rc;
    if ((e = hipMemcpyAsync(sk.data(), ctx->status.p, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "multi-key status");
    bool opened = false;
    for (uint32_t i = 0; i < n; i++) {
      sel[i] = st[i] == CE_ERR_AUTH && sk[i] == CE_OK;
      opened |= sel[i] != 0;
    }
    if (!opened) continue;
    if ((e = hipMemcpyAsync(c->d_refold2.p, sel.data(), n, hipMemcpyHostToDevice, ctx->stream)))
      return ctx->hip_fail(e, "multi-key mask");
    if ((rc = decode_only_resolving(c, da, n, c->d_refold2.as<uint8_t>()))) return rc;
    if ((e = hipMemcpyAsync(sk.data(), ctx->status.p, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "multi-key status");
    for (uint32_t i = 0; i < n; i++)
      if (sel[i]) st[i] = sk[i];  // CE_OK, or the decode's CE_ERR_DECODE / PT_* status
  }
  return CE_OK;
}

int ingest_ops_dev_once(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                        uint64_t blob_len, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                        const uint64_t* d_fv, int32_t* status_out, const AfterCommit* after_commit,
                        bool* merged_out, const uint64_t* shard_hi = nullptr) {
  if (merged_out) *merged_out = false;
  ce_ctx* ctx = c->ctx;
  // sharded (shard_hi): the gate is the agreed windows, and nothing is committed -- the batch
  // stays in d_batch for ce_core_pending_commit (cross-rank all-or-nothing)
  const bool sharded = shard_hi != nullptr;
  c->pending = false;
  if (!c->has_key) return ctx->fail(CE_ERR_NO_KEY, "no latest key");
  if (n == 0) return CE_OK;
  if (is_dotset_kind(c->kind))
    return ds_ingest_ops(c, d_blob, d_offs, n, blob_len, actors, m, d_fa, d_fv, status_out);
  hipError_t e;
  const KeyRef key = key_of(c);
  // writer actors (the op directories) get slots first: the version gate is keyed by them
  // (a repeated writer list -- the same shard every step -- reuses the previous lookup)
  std::vector<uint32_t> wslot;
  if (c->last_writers_gen == c->table_gen && c->last_writers.size() == 16ull * m &&
      std::memcmp(c->last_writers.data(), actors, 16ull * m) == 0) {
    wslot = c->last_wslot;
  } else {
    wslot.resize(m);
    const uint64_t gen0 = c->table_gen;
    for (uint32_t a = 0; a < m; a++) {
      Uuid u;
      std::memcpy(u.data(), actors + 16ull * a, 16);
      int rc = insert_actor(c, u, &wslot[a]);
      if (rc) return rc;
    }
    if (c->table_gen != gen0) refresh_slots(c, actors, m, &wslot);  // a growth moved them
    c->last_writers.assign(actors, actors + 16ull * m);
    c->last_wslot = wslot;
    c->last_writers_gen = c->table_gen;
  }
  int rc = table_upload(c);
  if (rc) return rc;
  if ((rc = ensure_supported(c))) return rc;
  if ((e = ctx->out.reserve(blob_len + 16ull * n + 128)) || (e = ctx->status.reserve(n * 4ull + 64)) ||
      (e = ctx->apply.reserve(n + 64)) || (e = ctx->refold.reserve(n + 64)) ||
      (e = c->d_refold2.reserve(n + 64)) || (e = ctx->miss.reserve(65536 * 16)) ||
      (e = c->d_gate.reserve(m * 32ull + 8ull * c->cap + 64)) ||
      (e = ctx->h_stage2.reserve(m * 32ull + 8ull * c->cap + 64)) ||
      (e = ctx->redo.reserve(n + 64)))
    return ctx->hip_fail(e, "ingest reserve");

  // expected versions per writer (next_op_versions.get, lib.rs:481) and the writers' slots ->
  // device in one copy.  Device gate block: e0 u64[m] | wslot u32[m] (8m bytes) | newnov u64[m]
  // | run_count u32[m] | run_first u32[m] | (with a compaction behind the ingest) the whole
  // pre-ingest next_op_versions u64[cap]; host stage: e0 | wslot | nov read back | zeros | nov
  uint64_t* he0 = ctx->h_stage2.as<uint64_t>();
  for (uint32_t a = 0; a < m; a++) he0[a] = c->nov[wslot[a]];
  std::memcpy(he0 + m, wslot.data(), m * 4ull);
  if (after_commit) std::memcpy(reinterpret_cast<uint8_t*>(he0) + 32ull * m, c->nov.data(), 8ull * c->cap);
  GateArgs ga{};
  ga.fa = d_fa;
  ga.fv = d_fv;
  ga.n = n;
  ga.m = m;
  uint8_t* gbase = c->d_gate.as<uint8_t>();
  ga.e0 = reinterpret_cast<const uint64_t*>(gbase);
  ga.newnov = reinterpret_cast<unsigned long long*>(gbase + 16ull * m);
  ga.run_count = reinterpret_cast<uint32_t*>(gbase + 24ull * m);
  ga.run_first = reinterpret_cast<uint32_t*>(gbase + 28ull * m);
  ga.flags = ctx->counters.as<uint32_t>() + 12;  // [12] not grouped, [13] first gap
  ga.apply = ctx->apply.as<uint8_t>();

  // the gate block (e0 | wslot, and with a compaction behind the ingest the pre-ingest
  // next_op_versions) read by the scratch fill itself from the mapped pinned stage: no DMA and
  // no cross-stream event before the gate (CE_GATE_DMA=1: the side-stream upload, for A/B)
  static const bool gate_dma = getenv("CE_GATE_DMA") != nullptr;
  const uint8_t* he0_dev = nullptr;
  if (!gate_dma) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, he0, 0) == hipSuccess) he0_dev = static_cast<const uint8_t*>(dp);
    else (void)hipGetLastError();
  }
  if (!he0_dev &&
      ((!ctx->side && (e = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking))) ||
       (!ctx->up_ev && (e = hipEventCreateWithFlags(&ctx->up_ev, hipEventDisableTiming))) ||
       (e = hipMemcpyAsync(gbase, he0, 12ull * m, hipMemcpyHostToDevice, ctx->side)) ||
       (after_commit && (e = hipMemcpyAsync(gbase + 32ull * m, reinterpret_cast<uint8_t*>(he0) + 32ull * m,
                                            8ull * c->cap, hipMemcpyHostToDevice, ctx->side))) ||
       (e = hipEventRecord(ctx->up_ev, ctx->side))))
    return ctx->hip_fail(e, "gate upload");

  // 1) GPU: scratch initialisation (one launch: counters, gate, batch state, miss / redo
  //    marks), device gate, setup (outer version, envelope, key schedule)
  static const bool gate_after_setup = getenv("CE_GATE_AFTER_SETUP") != nullptr;
  auto launch_gate_now = [&]() -> int {
    if (!he0_dev && (e = hipStreamWaitEvent(ctx->stream, ctx->up_ev, 0))) return ctx->hip_fail(e, "gate upload");
    const int t = ctx->tbegin("gate");
    if ((e = sharded ? launch_gate_window(ctx->stream, ga, shard_hi, ctx->counters.as<uint32_t>())
                     : launch_gate(ctx->stream, ga)))
      return ctx->hip_fail(e, "gate");
    ctx->tend(t);
    return CE_OK;
  };
  uint32_t ec;
  {
    FillArgs fl{};
    fl.r[0] = {reinterpret_cast<uint32_t*>(gbase + 16ull * m), 4ull * m, 0u};  // newnov, runs
    fl.r[1] = {c->d_batch.as<uint32_t>(), 2ull * c->cap, 0u};
    fl.r[2] = {ctx->refold.as<uint32_t>(), (n + 3ull) / 4, 0u};
    fl.r[3] = {ctx->redo.as<uint32_t>(), (n + 3ull) / 4, 0u};
    fl.n = 4;
    if (he0_dev) {
      fl.r[fl.n++] = {reinterpret_cast<uint32_t*>(gbase), 3ull * m, 0u, reinterpret_cast<const uint32_t*>(he0_dev)};
      if (after_commit)
        fl.r[fl.n++] = {reinterpret_cast<uint32_t*>(gbase + 32ull * m), 2ull * c->cap, 0u,
                        reinterpret_cast<const uint32_t*>(he0_dev + 32ull * m)};
    }
    // device_open's setup only; the fused kernel replaces its segment pass for small files.
    // The gate between the fill and the setup (it needs the filled gate block and the uploaded
    // e0, not the setup), so the setup runs straight into the fused kernel (CE_GATE_AFTER_SETUP:
    // the order before, for A/B)
    if (!gate_after_setup) {
      const std::function<int()> gate = launch_gate_now;
      int rr = device_open_setup(ctx, d_blob, d_offs, n, blob_len, true, key, ctx->status.as<int32_t>(),
                                 &ec, &fl, &gate);
      if (rr) return rr;
    } else {
      int rr = device_open_setup(ctx, d_blob, d_offs, n, blob_len, true, key, ctx->status.as<int32_t>(),
                                 &ec, &fl);
      if (rr) return rr;
    }
  }
  // the setup's counters (large-file count [9]) -> host behind an event: read while the fused
  // kernel runs, they decide whether the multi-page kernels are launched at all
  uint32_t* hsetup = ctx->h_counters.as<uint32_t>() + 32;
  // a one-wave kernel behind the setup writes its counters into the mapped pinned words with a
  // generation after them (no event marker or side-stream copy between the setup and the fused
  // kernel; CE_SETUP_EVENT=1: that older form, for A/B)
  static const bool setup_event = getenv("CE_SETUP_EVENT") != nullptr;
  uint32_t* hsetup_dev = nullptr;
  if (!setup_event) {
    void* dp = nullptr;
    if (hipHostGetDevicePointer(&dp, hsetup, 0) == hipSuccess) hsetup_dev = static_cast<uint32_t*>(dp);
    else (void)hipGetLastError();
  }
  const uint32_t gen = ++ctx->publish_gen ? ctx->publish_gen : ++ctx->publish_gen;  // never 0
  if (hsetup_dev) {
    if ((e = launch_publish_words(ctx->stream, ctx->counters.as<uint32_t>(), 16, hsetup_dev, gen)))
      return ctx->hip_fail(e, "setup counters");
  } else {
    if ((!ctx->setup_ev && (e = hipEventCreateWithFlags(&ctx->setup_ev, hipEventDisableTiming))) ||
        (!ctx->side_ev && (e = hipEventCreateWithFlags(&ctx->side_ev, hipEventDisableTiming))) ||
        (!ctx->side && (e = hipStreamCreateWithFlags(&ctx->side, hipStreamNonBlocking))))
      return ctx->hip_fail(e, "event");
    // on the side stream, behind the setup kernel: the main stream goes on to the gate and the
    // fused kernel without a copy between them
    if ((e = hipEventRecord(ctx->side_ev, ctx->stream)) || (e = hipStreamWaitEvent(ctx->side, ctx->side_ev, 0)) ||
        (e = hipMemcpyAsync(hsetup, ctx->counters.p, 64, hipMemcpyDeviceToHost, ctx->side)) ||
        (e = hipEventRecord(ctx->setup_ev, ctx->side)))
      return ctx->hip_fail(e, "setup counters");
  }
  bool setup_known = false;
  uint32_t n_large = 0;
  if (gate_after_setup) {
    const int rg = launch_gate_now();
    if (rg) return rg;
  }
  DecodeArgs da{};
  da.pt = ctx->out.as<uint8_t>();
  da.blob = d_blob;
  da.params = ctx->params.as<FileParams>();
  da.aux = ctx->poly_aux.as<PolyAux>();  // written by device_open_setup above
  da.status = ctx->status.as<int32_t>();
  da.n = n;
  da.supported = c->d_supported.as<uint8_t>();
  da.n_supported = (uint32_t)c->supported.size();
  da.apply = ctx->apply.as<uint8_t>();
  da.counters = ctx->counters.as<uint32_t>();
  da.miss_list = ctx->miss.as<uint4>();
  da.miss_cap = 65536;
  da.refold = ctx->refold.as<uint8_t>();
  da.table = c->d_table.as<ActorSlot>();
  da.mask = c->cap - 1;
  da.nil_actor = table_has_nil(c);
  da.batch = c->d_batch.as<unsigned long long>();
  da.large_list = ctx->large.as<uint32_t>();
#if CE_FUSED_DIAG  // diagnostics build (make prof -> libcrdtenc_prof.so)
  if (const char* ab = getenv("CE_ABLATE")) da.ablate = atoi(ab);
  const bool prof = getenv("CE_PROF") != nullptr;
#else
  const bool prof = false;
#endif
  static DevBuf& prof_buf = *new DevBuf;  // CE_PROF diagnostics (never freed): per-wave phase cycles
  if (prof) {
    if ((e = prof_buf.reserve(8ull * 8 * 65536)) || (e = hipMemsetAsync(prof_buf.p, 0, 8ull * 8 * 65536, ctx->stream)))
      return ctx->hip_fail(e, "prof");
    da.prof = prof_buf.as<unsigned long long>();
  }

  // 2) GPU: single-page files: open + decode + fold fused; larger files: segments + decode
  auto run_fold = [&](const uint8_t* only) -> int {
    da.only = only;
    da.large_only = 1;
    if (c->fused == 2 && c->files_per_wave != 1) {
      hipEvent_t t0, t1;
      (void)ctx->tlaunch("open_fold_small", &t0, &t1);
      if ((e = launch_open_fold_v2(ctx->stream, da, c->files_per_wave, t0, t1))) return ctx->hip_fail(e, "fused");
    } else {
      const int t = ctx->tbegin("open_fold_small");
      if ((e = launch_open_fold_small(ctx->stream, da, c->files_per_wave))) return ctx->hip_fail(e, "fused");
      ctx->tend(t);
    }
    if (!setup_known) {  // landed long ago: the fused kernel follows it
      if (hsetup_dev) {
        volatile const uint32_t* hp = hsetup;
        for (uint64_t i = 0; hp[16] != gen; i++) {
          if (i >= 64) sched_yield();
          if (i == (1ull << 22)) {  // (never expected) the stream's own wait, then the word must be there
            if ((e = hipStreamSynchronize(ctx->stream))) return ctx->hip_fail(e, "setup counters");
          } else if (i > (1ull << 22) && hp[16] != gen) {
            return ctx->fail(CE_ERR_DEVICE, "setup counters never published");
          }
        }
        std::atomic_thread_fence(std::memory_order_acquire);
      } else if ((e = hipEventSynchronize(ctx->setup_ev))) {
        return ctx->hip_fail(e, "setup counters");
      }
      n_large = hsetup[9];
      setup_known = true;
    }
    if (n_large == 0) return CE_OK;  // every file was single-page: nothing for the kernels below
    // decode inside the segment pass (CE_SEGDEC=0 or CE_SPLIT=1: the separate decode kernels
    // below; read per call, as CE_SPLIT)
    const char* sdv = getenv("CE_SEGDEC");
    const bool segdec = !(sdv && sdv[0] == '0') && !getenv("CE_SPLIT");
    if (!only) {
      SegScratch sc = segscratch(ctx, ec);
      if (segdec && (e = ctx->segrec.reserve((size_t)ec * 2 * 32))) return ctx->hip_fail(e, "segment records");
      int t = ctx->tbegin("segments_open");
      if ((e = segdec ? launch_segments_decode(ctx->stream, d_blob, ctx->out.as<uint8_t>(), da, sc,
                                               grid_waves_for(n + ec), ctx->segrec.as<uint4>())
                      : launch_segments(ctx->stream, false, d_blob, ctx->out.as<uint8_t>(), da.params, n,
                                        da.status, sc, grid_waves_for(n + ec), true)))
        return ctx->hip_fail(e, "segments");
      ctx->tend(t);
      t = ctx->tbegin("finalize_open");
      if ((e = launch_finalize_multi(ctx->stream, false, ctx->out.as<uint8_t>(), da.params, da.status, sc, n)))
        return ctx->hip_fail(e, "finalize");
      ctx->tend(t);
      if (segdec) {
        t = ctx->tbegin("decode");
        DecodeArgs rd = da;
        rd.redo = ctx->redo.as<uint8_t>();
        if ((e = launch_segdec_apply(ctx->stream, rd, sc, ctx->segrec.as<uint4>(), n_large)))
          return ctx->hip_fail(e, "decode");
        // files whose records did not prove out: the whole-file decode over the marked ones
        rd.only = rd.redo;
        if ((e = launch_decode_dots(ctx->stream, rd, grid_waves_for(n)))) return ctx->hip_fail(e, "decode");
        ctx->tend(t);
        return CE_OK;
      }
    }
    const int t = ctx->tbegin("decode");
    // CE_SPLIT=1: k_decode_split (measured slower on C4: 1.67 vs 1.36 ms)
    if (only || !getenv("CE_SPLIT")) {
      // counters[15]: the large-file list's pull index (k_decode_dots, large_only && !only),
      // zeroed with the counter block
      if ((e = launch_decode_dots(ctx->stream, da, grid_waves_for(n))))
        return ctx->hip_fail(e, "decode");
    } else {
      // every record a file's apply step reads is written by this batch's parts (no memset)
      if ((e = ctx->split.reserve((size_t)n_large * kSplitParts * 16))) return ctx->hip_fail(e, "split scratch");
      SplitScratch sp{ctx->split.as<uint4>()};
      if ((e = launch_decode_split(ctx->stream, da, sp, n_large))) return ctx->hip_fail(e, "decode");
    }
    ctx->tend(t);
    return CE_OK;
  };
  if ((rc = run_fold(nullptr))) return rc;
  // commit on the device unless the counters flag a slow path (k_merge_max_if), then one read
  // of the counters and of the gate's next_op_versions
  // (with a compaction behind the ingest, its first kernel does this commit)
  if (!sharded && !after_commit) {
    const int t = ctx->tbegin("merge");
    if ((e = launch_merge_max_if(ctx->stream, c->d_state.as<unsigned long long>(),
                                 c->d_batch.as<unsigned long long>(), c->cap,
                                 ctx->counters.as<uint32_t>())))
      return ctx->hip_fail(e, "merge");
    ctx->tend(t);
  }
  const uint8_t* host_tail = nullptr;
  if (after_commit) {  // the compaction, queued behind the commit (the writers' slots came with e0)
    NovApply na{reinterpret_cast<const uint32_t*>(gbase + 8ull * m),
                reinterpret_cast<const unsigned long long*>(gbase + 16ull * m), m,
                ctx->counters.as<uint32_t>()};
    na.nov_dev = reinterpret_cast<unsigned long long*>(gbase + 32ull * m);
    if (!sharded) {
      na.merge_dst = c->d_state.as<unsigned long long>();
      na.merge_src = c->d_batch.as<unsigned long long>();
      na.merge_n = c->cap;
    }
    if ((rc = (*after_commit)(na))) return rc;
    host_tail = na.host_tail;  // it downloads the counters and newnov with its own tail
  }
  // the gate's next_op_versions and the counter block, read back together at the end
  uint64_t* hnov = he0 + 2ull * m;
  if (!host_tail &&
      (e = hipMemcpyAsync(hnov, gbase + 16ull * m, m * 8ull, hipMemcpyDeviceToHost, ctx->stream)))
    return ctx->hip_fail(e, "nov");
  if (prof) {
    std::vector<unsigned long long> hp(8ull * 65536);
    if ((e = hipMemcpyAsync(hp.data(), prof_buf.p, hp.size() * 8, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "prof");
    double sum[7] = {0, 0, 0, 0, 0, 0, 0};
    uint32_t waves = 0;
    for (size_t w = 0; w < 65536; w++)
      if (hp[8 * w + 6]) {
        waves++;
        for (int i = 0; i < 7; i++) sum[i] += (double)hp[8 * w + i];
      }
    if (waves)
      // phase order: k_open_fold_small = params, chacha, xor_horner, tree_tag, decode prelude,
      // decode rounds; k_open_fold_v2 = setup, first block, middle blocks, last block,
      // tree_tag, decode
      fprintf(stderr, "CE_PROF waves %u iters/wave %.1f cycles/iter: p0 %.0f p1 %.0f p2 %.0f "
              "p3 %.0f p4 %.0f p5 %.0f\n", waves, sum[6] / waves,
              sum[0] / sum[6], sum[1] / sum[6], sum[2] / sum[6], sum[3] / sum[6], sum[4] / sum[6], sum[5] / sum[6]);
  }
  uint32_t* hc = ctx->h_counters.as<uint32_t>();
  if ((!host_tail && (e = hipMemcpyAsync(hc, ctx->counters.p, 64, hipMemcpyDeviceToHost, ctx->stream))) ||
      (e = ctx->sync_spin()))
    return ctx->hip_fail(e, "fold sync");
  if (host_tail) {
    std::memcpy(hc, host_tail + 8, 64);
    std::memcpy(hnov, host_tail + 72, 8ull * m);
  }
  const bool merged_on_device = !sharded && (hc[2] | hc[3] | hc[4] | hc[7] | hc[8] | hc[12]) == 0;
  if (sharded && (hc[10] & (kShardBad | kShardE0Mismatch)))
    return ctx->fail(CE_ERR_SHARD, hc[10] & kShardE0Mismatch
                                       ? "ranks started from different next_op_versions"
                                       : "a rank's batch breaks the partition contract: exact windows needed");
  if (merged_out) *merged_out = merged_on_device;
  if (hc[11]) c->path_counts["segdec_records"] += hc[11];
  if (hc[14]) c->path_counts["segdec_fallback"] += hc[14];

  // 3) batches outside the device gate's shape: host gate, fold again with its flags
  std::vector<uint64_t> expect(he0, he0 + m);
  uint32_t first_gap = hc[13] == 0xffffffffu ? n : hc[13];
  bool host_gated = false;
  if (hc[12]) {
    std::vector<uint32_t> fa(n);
    std::vector<uint64_t> fv(n);
    std::vector<uint8_t> ap(n);
    if ((e = hipMemcpyAsync(fa.data(), d_fa, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = hipMemcpyAsync(fv.data(), d_fv, n * 8ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "host gate");
    for (uint32_t i = 0; i < n; i++)
      if (fa[i] >= m) return ctx->fail(CE_ERR_INVALID_ARG, "file_actor out of range");
    first_gap = host_gate(fa.data(), fv.data(), n, &expect, ap.data());
    host_gated = true;
    if ((e = hipMemcpyAsync(ctx->apply.p, ap.data(), n, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemsetAsync(c->d_batch.p, 0, c->cap * 8ull, ctx->stream)) ||
        (e = hipMemsetAsync(c->d_refold2.p, 1, n, ctx->stream)) ||
        (e = hipMemsetAsync(ctx->refold.p, 0, n, ctx->stream)) ||
        (e = hipMemsetAsync(ctx->counters.as<uint32_t>() + 4, 0, 4, ctx->stream)))
      return ctx->hip_fail(e, "host gate");
    if ((rc = run_fold(c->d_refold2.as<uint8_t>()))) return rc;
    if ((e = hipMemcpyAsync(hc, ctx->counters.p, 64, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "fold sync");
  }

  // 4) misses: actors not in the table -> insert, upload, fold again the files that missed
  // (with CE_OPEN_MULTI_KEY an authentication failure may still be retried under another key,
  // so the files that did open must have their misses folded too)
  const bool may_retry = (c->flags & CE_OPEN_MULTI_KEY) && !c->alt_keys.empty();
  for (int round = 0; hc[4] != 0 && (hc[2] == 0 || may_retry) && hc[3] == 0 && hc[8] == 0; round++) {
    const uint32_t nm = std::min<uint32_t>(hc[4], 65536);
    std::vector<uint4> ml(nm);
    if ((e = hipMemcpyAsync(ml.data(), ctx->miss.p, nm * 16ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = hipMemcpyAsync(c->d_refold2.p, ctx->refold.p, n, hipMemcpyDeviceToDevice, ctx->stream)) ||
        (e = hipMemsetAsync(ctx->refold.p, 0, n, ctx->stream)) ||
        (e = hipMemsetAsync(ctx->counters.as<uint32_t>() + 4, 0, 4, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "miss");
    const uint32_t old_cap = c->cap;
    for (auto& x : ml) {
      Uuid u;
      std::memcpy(u.data(), &x, 16);
      uint32_t s;
      if ((rc = insert_actor(c, u, &s))) return rc;
    }
    if (c->cap != old_cap) {
      // slots moved: the partial batch state is stale -> fold everything again
      if ((e = hipMemsetAsync(c->d_batch.p, 0, c->cap * 8ull, ctx->stream)) ||
          (e = hipMemsetAsync(c->d_refold2.p, 1, n, ctx->stream)))
        return ctx->hip_fail(e, "miss");
    }
    if ((rc = table_upload(c))) return rc;
    for (uint32_t a = 0; a < m; a++) {
      Uuid u;
      std::memcpy(u.data(), actors + 16ull * a, 16);
      wslot[a] = c->slot_of[u];
    }
    da.table = c->d_table.as<ActorSlot>();
    da.mask = c->cap - 1;
    da.nil_actor = table_has_nil(c);
    da.batch = c->d_batch.as<unsigned long long>();
    if ((rc = run_fold(c->d_refold2.as<uint8_t>()))) return rc;
    if ((e = hipMemcpyAsync(hc, ctx->counters.p, 64, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "refold");
    if (round > 64) return ctx->fail(CE_ERR_DEVICE, "actor table did not converge");
  }

  // statuses: needed by the caller, for host-parse envelopes and to name the first failure
  // counters: [2] auth, [3] decode, [7] host-parse envelopes, [8] setup failures
  std::vector<int32_t> st;
  auto fetch_status = [&]() -> int {
    st.resize(n);
    if ((e = hipMemcpyAsync(st.data(), ctx->status.p, n * 4ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "status");
    return CE_OK;
  };
  const bool failed = hc[2] || hc[3] || hc[8];
  if (status_out || failed || hc[7]) {
    if ((rc = fetch_status())) return rc;
  }
  if (hc[7]) {
    if ((rc = resolve_host_parse(c, d_blob, d_offs, n, true))) return rc;
    std::vector<uint8_t> only(n, 0);
    for (uint32_t i = 0; i < n; i++) only[i] = st[i] == kStatusHostParse;
    if ((e = hipMemcpy(c->d_refold2.p, only.data(), n, hipMemcpyHostToDevice))) return ctx->hip_fail(e, "x");
    // misses go through the same insert / upload / fold-again loop as the fused path's
    if ((rc = decode_only_resolving(c, da, n, c->d_refold2.as<uint8_t>()))) return rc;
    if ((rc = fetch_status())) return rc;
  }
  if ((c->flags & CE_OPEN_MULTI_KEY) && !c->alt_keys.empty() && st.size() == n) {
    bool only_auth = true, any_auth = false;
    for (uint32_t i = 0; i < n; i++) {
      only_auth &= st[i] == CE_OK || st[i] == CE_ERR_AUTH;
      any_auth |= st[i] == CE_ERR_AUTH;
    }
    if (any_auth && only_auth && (rc = retry_alt_keys(c, da, d_blob, d_offs, n, blob_len, st))) return rc;
  }
  int first = CE_OK;
  if (st.size() == n) {
    for (uint32_t i = 0; i < n && first == CE_OK; i++)
      if (st[i] != CE_OK) first = st[i];
    if (status_out) std::memcpy(status_out, st.data(), n * 4ull);
  }
  if (first != CE_OK) return first;  // all-or-nothing: batch state discarded (lib.rs:497-514)

  // 5) commit: state = max(state, batch); next_op_versions from the gate
  if (sharded) {  // pending until ce_core_pending_commit: the windows' next_op_versions
    std::vector<uint64_t> nn(m);
    if ((e = hipMemcpyAsync(nn.data(), gbase + 16ull * m, m * 8ull, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "nov");
    c->pending_nov.clear();
    for (uint32_t a = 0; a < m; a++) {
      Uuid u;
      std::memcpy(u.data(), actors + 16ull * a, 16);
      c->pending_nov.push_back({u, std::max(expect[a], nn[a])});
    }
    c->pending = true;
    c->pending_gen = c->table_gen;
    return (hc[10] & kShardGap) ? CE_ERR_OP_VERSION : CE_OK;
  }
  if (merged_on_device) {
    for (uint32_t a = 0; a < m; a++) expect[a] = std::max(expect[a], hnov[a]);
  } else {
    const int t = ctx->tbegin("merge");
    if ((e = launch_merge_max(ctx->stream, c->d_state.as<unsigned long long>(),
                              c->d_batch.as<unsigned long long>(), c->cap)))
      return ctx->hip_fail(e, "merge");
    ctx->tend(t);
    if (!host_gated) {
      std::vector<uint64_t> nn(m);
      if ((e = hipMemcpyAsync(nn.data(), gbase + 16ull * m, m * 8ull, hipMemcpyDeviceToHost, ctx->stream)) ||
          (e = stream_wait(ctx->stream)))
        return ctx->hip_fail(e, "nov");
      for (uint32_t a = 0; a < m; a++) expect[a] = std::max(expect[a], nn[a]);
    } else if ((e = stream_wait(ctx->stream))) {
      return ctx->hip_fail(e, "merge");
    }
  }
  for (uint32_t a = 0; a < m; a++) c->nov[wslot[a]] = std::max(c->nov[wslot[a]], expect[a]);
  if (first_gap < n) {
    if (status_out) status_out[first_gap] = CE_ERR_OP_VERSION;
    return CE_ERR_OP_VERSION;
  }
  return CE_OK;
}

int ingest_ops_dev(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                   uint64_t blob_len, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                   const uint64_t* d_fv, int32_t* status_out, const AfterCommit* after_commit = nullptr,
                   bool* merged_out = nullptr, const uint64_t* shard_hi = nullptr) {
  for (int pass = 0;; pass++) {
    int rc = ingest_ops_dev_once(c, d_blob, d_offs, n, blob_len, actors, m, d_fa, d_fv, status_out,
                                 after_commit, merged_out, shard_hi);
    if (rc != kRestartIngest) return rc;
    if (pass > 8) return c->ctx->fail(CE_ERR_DEVICE, "actor table did not converge");
  }
}

int ingest_ops_dev_sharded(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                           uint64_t blob_len, const uint8_t* actors, uint32_t m, const uint32_t* d_fa,
                           const uint64_t* d_fv, const uint64_t* shard_hi, int32_t* status_out) {
  return ingest_ops_dev(c, d_blob, d_offs, n, blob_len, actors, m, d_fa, d_fv, status_out, nullptr,
                        nullptr, shard_hi);
}

// host metadata -> device, then ingest_ops_dev
int ingest_ops_hostmeta(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                        uint64_t blob_len, const uint8_t* actors, uint32_t m,
                        const uint32_t* file_actor, const uint64_t* file_version,
                        int32_t* status_out) {
  ce_ctx* ctx = c->ctx;
  for (uint32_t i = 0; i < n; i++)
    if (file_actor[i] >= m) return ctx->fail(CE_ERR_INVALID_ARG, "file_actor out of range");
  hipError_t e;
  if ((e = c->d_meta.reserve(n * 12ull + 64))) return ctx->hip_fail(e, "meta");
  uint8_t* mb = c->d_meta.as<uint8_t>();
  if ((e = hipMemcpyAsync(mb, file_version, n * 8ull, hipMemcpyHostToDevice, ctx->stream)) ||
      (e = hipMemcpyAsync(mb + 8ull * n, file_actor, n * 4ull, hipMemcpyHostToDevice, ctx->stream)) ||
      (e = stream_wait(ctx->stream)))
    return ctx->hip_fail(e, "meta upload");
  return ingest_ops_dev(c, d_blob, d_offs, n, blob_len, actors, m,
                        reinterpret_cast<const uint32_t*>(mb + 8ull * n),
                        reinterpret_cast<const uint64_t*>(mb), status_out);
}

int ingest_states_dev(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n, uint64_t blen,
                      int32_t* status_out);

// Core::read_remote_states after Storage::load_states (lib.rs:425-466)
// files (optional): per-file host buffers instead of one blob (ce_core_ingest_states_iov),
// uploaded through the pinned staging ring
int ingest_states_host(ce_core* c, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                       int32_t* status_out, const uint8_t* const* files = nullptr) {
  ce_ctx* ctx = c->ctx;
  if (!c->has_key) return ctx->fail(CE_ERR_NO_KEY, "no latest key");
  if (n == 0) return CE_OK;
  const uint64_t blen = offs[n];
  hipError_t e;
  if ((e = ctx->blob.reserve(blen + 64)) || (e = ctx->offs.reserve((n + 1) * 8ull)) ||
      (e = ctx->out.reserve(blen + 16ull * n + 128)) || (e = ctx->status.reserve(n * 4ull + 64)))
    return ctx->hip_fail(e, "states reserve");
  if (files) {
    int rc = stage_host_batch(ctx, files, offs, n);
    if (rc) return rc;
  } else if ((e = hipMemcpyAsync(ctx->blob.p, blob, blen, hipMemcpyHostToDevice, ctx->stream)) ||
             (e = hipMemcpyAsync(ctx->offs.p, offs, (n + 1) * 8ull, hipMemcpyHostToDevice, ctx->stream))) {
    return ctx->hip_fail(e, "states upload");
  }
  return ingest_states_dev(c, ctx->blob.as<uint8_t>(), ctx->offs.as<uint64_t>(), n, blen, status_out);
}

// read_remote_states over state files resident in HBM (d_blob / d_offs, n + 1 offsets)
int ingest_states_dev(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n, uint64_t blen,
                      int32_t* status_out) {
  ce_ctx* ctx = c->ctx;
  if (!c->has_key) return ctx->fail(CE_ERR_NO_KEY, "no latest key");
  if (n == 0) return CE_OK;
  hipError_t e;
  if ((e = ctx->out.reserve(blen + 16ull * n + 128)) || (e = ctx->status.reserve(n * 4ull + 64)))
    return ctx->hip_fail(e, "states reserve");
  HostPhase hp("states: open + download");
  int rc = device_open(ctx, d_blob, d_offs, n, blen, true, key_of(c), ctx->out.as<uint8_t>(),
                       ctx->status.as<int32_t>(), false);
  if (rc) return rc;
  // one download for what the host reads per file (k_state_heads, 32 B each into pinned
  // memory): status, clear length, plaintext offset and data version -- per-file copies into
  // pageable memory each cost a blit dispatch and a staging wait on the box
  if ((e = ctx->heads.reserve(32ull * n + 64)) || (e = ctx->h_heads.reserve(32ull * n + 64)))
    return ctx->hip_fail(e, "states heads");
  const uint8_t* hh = ctx->h_heads.as<uint8_t>();
  std::vector<int32_t> st(n);
  auto read_heads = [&]() -> hipError_t {
    hipError_t e2;
    if ((e2 = launch_state_heads(ctx->stream, ctx->params.as<FileParams>(), ctx->status.as<int32_t>(),
                                 ctx->out.as<uint8_t>(), n, ctx->heads.as<uint8_t>())) ||
        (e2 = hipMemcpyAsync(ctx->h_heads.p, ctx->heads.p, 32ull * n, hipMemcpyDeviceToHost, ctx->stream)) ||
        (e2 = stream_wait(ctx->stream)))
      return e2;
    for (uint32_t i = 0; i < n; i++) std::memcpy(&st[i], hh + 32ull * i, 4);
    return hipSuccess;
  };
  if ((e = read_heads())) return ctx->hip_fail(e, "states heads");
  // the host has waited for the device: a previous compaction's download can go now
  if (is_dotset_kind(c->kind) && (rc = ds_async_kick(c, false))) return rc;
  for (uint32_t i = 0; i < n; i++)
    if (st[i] == kStatusHostParse) {
      if ((rc = resolve_host_parse(c, d_blob, d_offs, n, true))) return rc;
      if ((e = read_heads())) return ctx->hip_fail(e, "states heads");
      break;
    }
  std::vector<FileParams> P(n);
  if (c->kind == CE_STATE_ORSWOT && !getenv("CE_HOST_STATES")) {
    // plaintexts stay in HBM: the device reader decodes canonical states (ce_dotset_io.hip)
    std::vector<uint64_t> off(n, 0), len(n, 0);
    for (uint32_t i = 0; i < n; i++) {
      if (st[i] != CE_OK) continue;
      const uint8_t* h = hh + 32ull * i;
      uint32_t plen;
      uint64_t out_off;
      std::memcpy(&plen, h + 4, 4);
      std::memcpy(&out_off, h + 8, 8);
      if (plen < 16) { st[i] = CE_ERR_PT_LEN; continue; }
      off[i] = out_off + 16;
      len[i] = plen - 16;
      Uuid v;
      std::memcpy(v.data(), h + 16, 16);
      if (!std::binary_search(c->supported.begin(), c->supported.end(), v)) st[i] = CE_ERR_PT_VERSION;
    }
    return ds_merge_states_device(c, ctx->out.as<uint8_t>(), off, len, st.data(), status_out);
  }
  std::vector<uint8_t> out(blen + 16ull * n + 64);
  if ((e = hipMemcpyAsync(P.data(), ctx->params.p, n * sizeof(FileParams), hipMemcpyDeviceToHost,
                          ctx->stream)) ||
      (e = hipMemcpyAsync(out.data(), ctx->out.p, blen + 16ull * n, hipMemcpyDeviceToHost, ctx->stream)) ||
      (e = stream_wait(ctx->stream)))
    return ctx->hip_fail(e, "states download");
  if (is_dotset_kind(c->kind)) {
    std::vector<std::pair<const uint8_t*, size_t>> sws(n, {nullptr, 0});
    for (uint32_t i = 0; i < n; i++) {
      if (st[i] != CE_OK) continue;
      const uint8_t* pt = out.data() + P[i].out_off;
      const uint32_t len = P[i].len;
      if (len < 16) { st[i] = CE_ERR_PT_LEN; continue; }
      Uuid v;
      std::memcpy(v.data(), pt, 16);
      if (!std::binary_search(c->supported.begin(), c->supported.end(), v)) { st[i] = CE_ERR_PT_VERSION; continue; }
      sws[i] = {pt + 16, len - 16};
    }
    return ds_merge_states(c, sws, st.data(), status_out);
  }
  // host pass: StateWrapper msgpack -> dots (north star: "host pass that flattens decoded
  // ops/states into columnar arrays")
  std::vector<Dots> novs(n), sts(n);
  int first = CE_OK;
  for (uint32_t i = 0; i < n; i++) {
    if (st[i] == CE_OK) {
      const uint8_t* pt = out.data() + P[i].out_off;
      const uint32_t len = P[i].len;
      if (len < 16) st[i] = CE_ERR_PT_LEN;
      else {
        Uuid v;
        std::memcpy(v.data(), pt, 16);
        if (!std::binary_search(c->supported.begin(), c->supported.end(), v)) st[i] = CE_ERR_PT_VERSION;
        else if (!read_state_wrapper(pt + 16, len - 16, c->kind, &novs[i], &sts[i]))
          st[i] = CE_ERR_DECODE;
      }
    }
    if (st[i] != CE_OK && first == CE_OK) first = st[i];
  }
  if (status_out) std::memcpy(status_out, st.data(), n * 4ull);
  if (first != CE_OK) return first;
  // fold (lib.rs:458-466): state.merge(sw.state); next_op_versions.merge(sw.next_op_versions)
  Dots all;
  for (uint32_t i = 0; i < n; i++) all.insert(all.end(), sts[i].begin(), sts[i].end());
  if ((rc = merge_dots_host(c, all))) return rc;
  for (uint32_t i = 0; i < n; i++)
    for (auto& d : novs[i]) {
      uint32_t s;
      if ((rc = insert_actor(c, d.first, &s))) return rc;
      c->nov[s] = std::max(c->nov[s], d.second);
    }
  return table_upload(c);
}

int read_remote(ce_core* c) {
  if (!c->storage) return c->ctx->fail(CE_ERR_INVALID_ARG, "core opened without storage");
  // read_remote_states (lib.rs:401-469)
  std::vector<std::string> names;
  int rc = storage_list_states_vec(c->storage, &names);
  if (rc) return c->ctx->fail(rc, "failed getting state entry names while reading remote states");
  std::vector<std::string> to_read;
  for (auto& nm : names)
    if (!c->read_states.count(nm)) to_read.push_back(nm);
  if (!to_read.empty()) {
    if (!c->has_key) return c->ctx->fail(CE_ERR_NO_KEY, "no latest key");
    std::vector<uint8_t> blob;
    std::vector<uint64_t> offs{0};
    for (auto& nm : to_read) {
      std::vector<uint8_t> f;
      if ((rc = storage_read_state(c->storage, nm, &f))) return c->ctx->fail(rc, "failed loading state content");
      blob.insert(blob.end(), f.begin(), f.end());
      offs.push_back(blob.size());
    }
    rc = ingest_states_host(c, blob.data(), offs.data(), (uint32_t)to_read.size(), nullptr);
    if (rc) return rc;
    for (auto& nm : to_read) c->read_states.insert(nm);
  }
  // read_remote_ops (lib.rs:471-547)
  std::vector<Uuid> actors;
  if ((rc = storage_list_op_actors_vec(c->storage, &actors))) return c->ctx->fail(rc, "failed getting op actor entries");
  if (actors.empty()) return CE_OK;
  if (!c->has_key) return c->ctx->fail(CE_ERR_NO_KEY, "no latest key");
  std::vector<uint64_t> first(actors.size());
  for (size_t a = 0; a < actors.size(); a++) {
    auto it = c->slot_of.find(actors[a]);
    first[a] = it == c->slot_of.end() ? 0 : c->nov[it->second];
  }
  std::vector<uint8_t> blob;
  std::vector<uint64_t> offs, vers;
  std::vector<uint32_t> aidx;
  if ((rc = storage_load_ops_vec(c->storage, actors, first, &blob, &offs, &aidx, &vers)))
    return c->ctx->fail(rc, "failed loading ops");
  const uint32_t n = (uint32_t)aidx.size();
  if (n == 0) return CE_OK;
  ce_ctx* ctx = c->ctx;
  hipError_t e;
  if ((e = ctx->blob.reserve(blob.size() + 64)) || (e = ctx->offs.reserve((n + 1) * 8ull)))
    return ctx->hip_fail(e, "ops reserve");
  if ((e = hipMemcpyAsync(ctx->blob.p, blob.data(), blob.size(), hipMemcpyHostToDevice, ctx->stream)) ||
      (e = hipMemcpyAsync(ctx->offs.p, offs.data(), (n + 1) * 8ull, hipMemcpyHostToDevice, ctx->stream)) ||
      (e = stream_wait(ctx->stream)))
    return ctx->hip_fail(e, "ops upload");
  std::vector<uint8_t> ab(actors.size() * 16);
  for (size_t a = 0; a < actors.size(); a++) std::memcpy(ab.data() + 16 * a, actors[a].data(), 16);
  return ingest_ops_hostmeta(c, ctx->blob.as<uint8_t>(), ctx->offs.as<uint64_t>(), n, blob.size(),
                             ab.data(), (uint32_t)actors.size(), aidx.data(), vers.data(), nullptr);
}

// compaction of a VClock / GCounter state without leaving the device: the StateWrapper is
// serialized from the dense arrays (k_serialize_vclock) into the seal's input, sealed, and only
// the sealed file comes back.  Same bytes as serialize_state + seal_one.
//   compact_enqueue: everything up to the download into x->h_stage, on x's stream (no sync).
//     With `na`, next_op_versions of the ingest still in flight is folded in on the device
//     (k_nov_apply, skipped exactly when that ingest's merge is) -- the host nov is then the
//     pre-ingest one.
//   compact_finish: after the stream has been synchronised, the file from the staging buffer.
struct CompactPending {
  uint64_t U = 0, total_max = 0;
  const uint8_t* tail = nullptr;  // pinned host: [clear length | counters | newnov] after sync
  bool to_sink = false;           // the file went straight into the caller's buffer (c->sink)
};

int compact_enqueue(ce_core* c, ce_ctx* x, const uint8_t* nonce, NovApply* na, CompactPending* pend) {
  const KeyRef key = key_of(c);
  if (int32_t ks = key_status(key)) return x->fail(ks, "key rejected");
  const bool ingest_fmt = (c->flags & CE_COMPACT_INGEST_FORMAT) != 0;
  // readable by read_remote_states: CURRENT_VERSION || encrypt(data_version || state); else
  // exactly what Core::compact writes: VersionBytes(current_data_version, encrypt(state))
  const uint8_t* outer = ingest_fmt ? kCoreVersion : c->current_data_version.data();
  ensure_sorted(c);
  const uint32_t k = (uint32_t)c->sorted_slots.size();
  int rc = table_upload(c);  // the serializer reads the UUIDs from the device table
  if (rc) return rc;
  hipError_t e;
  if (c->d_sorted_gen != c->sorted_gen) {
    if ((e = c->d_sorted.reserve(4ull * k + 64)) ||
        (k && (e = hipMemcpyAsync(c->d_sorted.p, c->sorted_slots.data(), 4ull * k, hipMemcpyHostToDevice,
                                  x->stream))) ||
        (e = stream_wait(x->stream)))
      return x->hip_fail(e, "sorted slots");
    c->d_sorted_gen = c->sorted_gen;
  }
  const uint64_t U = vclock_ser_bound(k);             // clear length bound (prefix included)
  const uint64_t A = (U + 255) & ~255ull;              // small arguments after the clear text
  const uint64_t total_max = 16 + sealed_len(U);
  const uint64_t T = (total_max + 255) & ~255ull;      // the packed tail after the file bound
  const uint32_t m = na ? na->m : 0;
  const uint64_t tail_bytes = 72 + 8ull * m;
  const uint64_t nov_bytes = 8ull * c->cap;
  uint32_t* seal_counters = ctx_counters(x);
  if (!seal_counters || (e = x->blob.reserve(A + 128)) || (e = x->out.reserve(T + tail_bytes + 64)) ||
      (e = x->h_stage.reserve(std::max<uint64_t>(T + tail_bytes + 64, 128 + nov_bytes))) ||
      (e = c->d_tmp.reserve(nov_bytes)))
    return x->hip_fail(e ? e : hipErrorOutOfMemory, "compact reserve");
  uint8_t* hs = x->h_stage.as<uint8_t>();
  uint8_t* db = x->blob.as<uint8_t>();
  // next_op_versions on the device: with `na` the pre-ingest copy the ingest uploaded with its
  // gate block (newnov applied below, in place), else uploaded here
  unsigned long long* nov = c->d_tmp.as<unsigned long long>();
  if (na && na->nov_dev) {
    nov = na->nov_dev;
  } else {
    std::memcpy(hs + 128, c->nov.data(), nov_bytes);
    if ((e = hipMemcpyAsync(nov, hs + 128, nov_bytes, hipMemcpyHostToDevice, x->stream)))
      return x->hip_fail(e, "compact upload");
  }
  CompactArgs ca;
  if (nonce) std::memcpy(ca.nonce, nonce, 24);
  else os_random(ca.nonce, 24);
  std::memcpy(ca.outer, outer, 16);
  std::memcpy(ca.prefix, c->current_data_version.data(), 16);
  // args at db + A: [offs(2) | out_offs(1) | nonce(24) | outer(16) | prefix16(16)]
  if ((e = launch_compact_prologue(x->stream, db + A, ca, seal_counters, nov, na ? na->wslot : nullptr,
                                   na ? na->newnov : nullptr, m, na ? na->counters : nullptr,
                                   na ? na->merge_dst : nullptr, na ? na->merge_src : nullptr,
                                   na ? na->merge_n : 0u)))
    return x->hip_fail(e, "compact prologue");
  auto* d_offs = reinterpret_cast<unsigned long long*>(db + A);
  if ((e = launch_serialize_vclock(x->stream, nov, c->d_state.as<unsigned long long>(), c->d_sorted.as<uint32_t>(),
                                   k, c->d_table.as<ActorSlot>(), c->kind == CE_STATE_GCOUNTER,
                                   ingest_fmt ? db + A + 64 : nullptr, db, d_offs)))
    return x->hip_fail(e, "serialize");
  rc = device_seal(x, db, reinterpret_cast<const uint64_t*>(d_offs), 1, U, db + A + 48, db + A + 24,
                   x->out.as<uint8_t>(), reinterpret_cast<const uint64_t*>(db + A + 16), key, true);
  if (rc) return rc;
  // the tail (clear length, and with `na` the ingest's counters and newnov) packed behind the file
  uint8_t* dtail = x->out.as<uint8_t>() + T;
  if ((e = launch_tail_pack(x->stream, dtail, reinterpret_cast<const unsigned long long*>(db + A + 8),
                            na ? na->counters : seal_counters, na ? na->newnov : nullptr, m)))
    return x->hip_fail(e, "tail pack");
  // downloads: the file straight into the caller's buffer when it has room (compact_into), the
  // tail beside it; else file and tail in one copy
  pend->to_sink = c->sink && c->sink_cap >= total_max;
  if (pend->to_sink && c->sink_cap >= T + tail_bytes) {  // room for the tail too: one copy
    if ((e = hipMemcpyAsync(c->sink, x->out.p, T + tail_bytes, hipMemcpyDeviceToHost, x->stream)))
      return x->hip_fail(e, "compact download");
    pend->tail = c->sink + T;
  } else if (pend->to_sink) {
    if ((e = hipMemcpyAsync(c->sink, x->out.p, total_max, hipMemcpyDeviceToHost, x->stream)) ||
        (e = hipMemcpyAsync(hs, dtail, tail_bytes, hipMemcpyDeviceToHost, x->stream)))
      return x->hip_fail(e, "compact download");
    pend->tail = hs;
  } else {
    if ((e = hipMemcpyAsync(hs, x->out.p, T + tail_bytes, hipMemcpyDeviceToHost, x->stream)))
      return x->hip_fail(e, "compact download");
    pend->tail = hs + T;
  }
  if (na) na->host_tail = pend->tail;
  pend->U = U;
  pend->total_max = total_max;
  return CE_OK;
}

int compact_finish(ce_core* c, ce_ctx* x, const CompactPending& pend, std::vector<uint8_t>* file) {
  uint64_t clear_len;
  std::memcpy(&clear_len, pend.tail, 8);
  if (clear_len > pend.U) return x->fail(CE_ERR_DEVICE, "serializer overran its bound");
  const uint64_t total = 16 + sealed_len(clear_len);
  if (pend.to_sink) {
    c->sink_len = total;
    file->clear();
    return CE_OK;
  }
  file->resize(total);
  std::memcpy(file->data(), x->h_stage.as<uint8_t>(), total);
  return CE_OK;
}

int compact_device(ce_core* c, const uint8_t* nonce, std::vector<uint8_t>* file) {
  CompactPending pend;
  int rc = compact_enqueue(c, c->ctx, nonce, nullptr, &pend);
  if (rc) return rc;
  hipError_t e;
  if ((e = stream_wait(c->ctx->stream))) return c->ctx->hip_fail(e, "compact sync");
  return compact_finish(c, c->ctx, pend, file);
}

// clear text + file of a compaction (lib.rs:335-360)
int compact_bytes(ce_core* c, const uint8_t* nonce, std::vector<uint8_t>* file) {
  HostPhase hp("compact_bytes");
  if (!c->has_key) return c->ctx->fail(CE_ERR_NO_KEY, "no latest key");
  if (!is_dotset_kind(c->kind) && !c->host_compact) return compact_device(c, nonce, file);
  if (c->kind == CE_STATE_ORSWOT && !c->host_compact) {
    // entries serialized, sealed and downloaded once on the device (ce_dotset_io.hip)
    const bool ingest_fmt = (c->flags & CE_COMPACT_INGEST_FORMAT) != 0;
    return ds_compact_device(c, c->ctx, ingest_fmt ? kCoreVersion : c->current_data_version.data(),
                             ingest_fmt ? c->current_data_version.data() : nullptr, nonce, key_of(c), file);
  }
  std::vector<uint8_t>& clear = c->ser_buf;
  int rc = serialize_state(c, &clear);
  if (rc) return rc;
  HostPhase hs("compact: seal");
  if (c->flags & CE_COMPACT_INGEST_FORMAT)  // readable by read_remote_states: CURRENT_VERSION ||
    return seal_one(c->ctx, key_of(c), kCoreVersion, nonce, clear.data(), clear.size(), file,
                    c->current_data_version.data());  // encrypt(data_version || state)
  // exactly what Core::compact writes: VersionBytes(current_data_version, encrypt(state))
  return seal_one(c->ctx, key_of(c), c->current_data_version.data(), nonce, clear.data(),
                  clear.size(), file);
}

}  // namespace ce

extern "C" {

int ce_core_open(ce_ctx* ctx, const ce_open_options* o, ce_core** out) {
  if (!ctx || !o || !out || !o->current_data_version || (o->n_supported && !o->supported_data_versions))
    return CE_ERR_INVALID_ARG;
  if (o->state_kind != CE_STATE_VCLOCK && o->state_kind != CE_STATE_GCOUNTER &&
      !is_dotset_kind(o->state_kind))
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(ctx->mu);
  (void)hipSetDevice(ctx->device);
  ce_core* c = new ce_core();
  c->ctx = ctx;
  c->kind = o->state_kind;
  if (const char* fw = getenv("CE_FILES_PER_WAVE")) {
    const int v = atoi(fw);
    if (v == 1 || v == 2 || v == 4) c->files_per_wave = v;
  }
  if (const char* fu = getenv("CE_FUSED")) {
    const int v = atoi(fu);
    if (v == 1 || v == 2) c->fused = v;
  }
  if (const char* hc = getenv("CE_HOST_COMPACT")) c->host_compact = atoi(hc) != 0;
  c->flags = o->flags;
  std::memcpy(c->current_data_version.data(), o->current_data_version, 16);
  for (size_t i = 0; i < o->n_supported; i++) {
    Uuid u;
    std::memcpy(u.data(), o->supported_data_versions + 16 * i, 16);
    c->supported.push_back(u);
  }
  std::sort(c->supported.begin(), c->supported.end());
  int rc = table_init(c, 8192);
  if (rc) { delete c; return rc; }
  if (is_dotset_kind(c->kind) && (rc = ds_init(c))) { ce_core_close(c); return rc; }
  if (o->local_path || o->remote_path) {
    if (!o->local_path || !o->remote_path || o->local_path[0] != '/' || o->remote_path[0] != '/') {
      delete c;
      return CE_ERR_INVALID_ARG;
    }
    c->storage = storage_new(o->local_path, o->remote_path);
    // load_local_meta (lib.rs:250-278)
    std::vector<uint8_t> lm;
    bool missing = false;
    if ((rc = storage_load_local_meta(c->storage, &lm, &missing))) { ce_core_close(c); return rc; }
    if (!missing) {
      if (lm.size() < 16 || std::memcmp(lm.data(), kCoreVersion, 16) != 0) {
        ce_core_close(c);
        return lm.size() < 16 ? CE_ERR_OUTER_LEN : CE_ERR_OUTER_VERSION;
      }
      Rd r{lm.data() + 16, lm.size() - 16, 0};
      bool ok = read_struct(r, {"local_actor_id"}, [&](int, Rd& q) {
        uint64_t off;
        if (!rd_uuid(q, &off)) return false;
        std::memcpy(c->local_actor.data(), q.p + off, 16);
        return true;
      });
      if (!ok) { ce_core_close(c); return CE_ERR_DECODE; }
    } else {
      if (!(o->flags & CE_OPEN_CREATE)) { ce_core_close(c); return CE_ERR_NO_LOCAL_META; }
      c->local_actor = uuid_v4();
      Wr w;
      w.b.assign(kCoreVersion, kCoreVersion + 16);  // VersionBytes(CURRENT_VERSION, ..)
      w.map(1);
      w.str("local_actor_id");
      w.bin(c->local_actor.data(), 16);
      if ((rc = storage_store_local_meta(c->storage, w.b.data(), w.b.size()))) { ce_core_close(c); return rc; }
    }
  } else {
    c->local_actor = uuid_v4();
  }
  if ((rc = table_upload(c))) { ce_core_close(c); return rc; }
  *out = c;
  return CE_OK;
}

void ce_core_close(ce_core* c) {
  if (!c) return;
  if (c->ctx) (void)hipStreamSynchronize(c->ctx->stream);
  c->pend = false;  // a download not enqueued yet is dropped (its buffer may be gone with the core)
  if (c->copy_stream) {
    (void)hipStreamSynchronize(c->copy_stream);
    (void)hipStreamDestroy(c->copy_stream);
  }
  for (hipEvent_t ev : c->copy_ev)
    if (ev) (void)hipEventDestroy(ev);
  for (uint32_t k = 0; k < ce_core::kAsyncSlots; k++)
    if (c->copy_sig[k].handle) {
      ce::dma_wait(c->copy_sig[k]);
      ce::dma_signal_destroy(c->copy_sig[k]);
    }
  if (c->seal_ev) (void)hipEventDestroy(c->seal_ev);
  delete c->storage;
  delete c->aux;
  ds_free(c->ds);
  delete c;
}

int ce_core_set_latest_key(ce_core* c, const uint8_t key_version[16], const uint8_t* key,
                           size_t key_len) {
  if (!c || !key_version || (key_len && !key)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  std::memcpy(c->key_version, key_version, 16);
  c->key.assign(key, key + key_len);
  c->has_key = true;
  c->alt_keys.clear();
  return CE_OK;
}

int ce_core_info_actor(ce_core* c, uint8_t out[16]) {
  if (!c || !out) return CE_ERR_INVALID_ARG;
  std::memcpy(out, c->local_actor.data(), 16);
  return CE_OK;
}

int ce_core_state_bytes(ce_core* c, ce_buf* out) {
  if (!c || !out) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  std::vector<uint8_t> b;
  int rc = serialize_state(c, &b);
  if (rc) return rc;
  out->data = (uint8_t*)malloc(b.size() ? b.size() : 1);
  std::memcpy(out->data, b.data(), b.size());
  out->len = b.size();
  return CE_OK;
}

int ce_core_ingest_ops(ce_core* c, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                       const uint8_t* actors, uint32_t m, const uint32_t* file_actor,
                       const uint64_t* file_version, int32_t* status) {
  if (!c || (n && (!blob || !offs || !actors || !file_actor || !file_version))) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (n == 0) return CE_OK;
  ce_ctx* ctx = c->ctx;
  // the blob goes up in chunks through pinned staging (ce_upload.cpp), ordered on the stream
  std::vector<const uint8_t*> fp(n);
  for (uint32_t i = 0; i < n; i++) fp[i] = blob + offs[i];
  std::vector<uint64_t> rel(offs, offs + n + 1);
  for (auto& x : rel) x -= offs[0];
  int rc = stage_host_batch(ctx, fp.data(), rel.data(), n);
  if (rc) return rc;
  return ingest_ops_hostmeta(c, ctx->blob.as<uint8_t>(), ctx->offs.as<uint64_t>(), n, rel[n], actors,
                             m, file_actor, file_version, status);
}

static int iov_offsets(const size_t* lens, uint32_t n, std::vector<uint64_t>* offs) {
  offs->resize(n + 1);
  (*offs)[0] = 0;
  for (uint32_t i = 0; i < n; i++) (*offs)[i + 1] = (*offs)[i] + lens[i];
  return CE_OK;
}

int ce_core_ingest_ops_iov(ce_core* c, const uint8_t* const* files, const size_t* lens, uint32_t n,
                           const uint8_t* actors, uint32_t m, const uint32_t* file_actor,
                           const uint64_t* file_version, int32_t* status) {
  if (!c || (n && (!files || !lens || !actors || !file_actor || !file_version))) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (n == 0) return CE_OK;
  std::vector<uint64_t> offs;
  iov_offsets(lens, n, &offs);
  int rc = stage_host_batch(c->ctx, files, offs.data(), n);
  if (rc) return rc;
  return ingest_ops_hostmeta(c, c->ctx->blob.as<uint8_t>(), c->ctx->offs.as<uint64_t>(), n, offs[n],
                             actors, m, file_actor, file_version, status);
}

int ce_core_ingest_ops_device(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs,
                              uint32_t n, uint64_t blob_len, const uint8_t* actors, uint32_t m,
                              const uint32_t* d_file_actor, const uint64_t* d_file_version,
                              int32_t* status) {
  if (!c || (n && (!d_blob || !d_offs || !actors || !d_file_actor || !d_file_version)))
    return CE_ERR_INVALID_ARG;
  HostPhase hp("ingest_ops_device (all)");
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  return ingest_ops_dev(c, d_blob, d_offs, n, blob_len, actors, m, d_file_actor, d_file_version,
                        status);
}

// Core::compact (lib.rs:332-380) over op files resident in HBM: read_remote_ops, then the
// compaction output.  The compaction (nov fold, serialize, seal, download) is enqueued behind
// the ingest's device commit on the aux context's buffers, so one host synchronisation covers
// both; when the ingest leaves its fast path the speculative file is dropped and the compaction
// runs again from the committed host state.
}  // extern "C"

namespace ce {
// Core::compact over a batch in HBM (shared by ce_core_compact_ops_device[_into]): the file ends
// up in c->sink when the caller gave one with room (*out = sink, c->sink_len), else in
// c->file_buf.  The caller holds the context lock.
static int compact_ops_device_impl(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                                   uint64_t blob_len, const uint8_t* actors, uint32_t m,
                                   const uint32_t* d_file_actor, const uint64_t* d_file_version,
                                   const uint8_t* nonce, const uint8_t** out, size_t* out_len,
                                   char name_out[64]) {
  if (!c->has_key) return c->ctx->fail(CE_ERR_NO_KEY, "no latest key");
  std::vector<uint8_t>& f = c->file_buf;
  int rc;
  bool merged = false;
  const bool spec = !is_dotset_kind(c->kind) && !c->host_compact && n > 0;
  ce_ctx* x = aux_ctx(c);  // same stream: the compaction is ordered behind the ingest
  CompactPending pend;
  uint8_t nb[24];  // one nonce for the speculative and (if needed) the repeated compaction
  if (nonce) std::memcpy(nb, nonce, 24);
  else os_random(nb, 24);
  c->sink_len = 0;
  const AfterCommit hook = [&](NovApply& na) { return compact_enqueue(c, x, nb, &na, &pend); };
  rc = ingest_ops_dev(c, d_blob, d_offs, n, blob_len, actors, m, d_file_actor, d_file_version, nullptr,
                      spec ? &hook : nullptr, &merged);
  if (rc) {
    if (spec) (void)hipStreamSynchronize(c->ctx->stream);  // nothing left in flight on x's buffers
    return rc;  // read_remote's error: compact writes nothing (lib.rs:333)
  }
  if (spec && merged) rc = compact_finish(c, x, pend, &f);
  else rc = compact_bytes(c, nb, &f);
  if (rc) return rc;
  if (c->sink_len) {
    *out = c->sink;
    *out_len = c->sink_len;
  } else {
    *out = f.data();
    *out_len = f.size();
  }
  if (name_out) {
    uint8_t h[32];
    sha3_256(*out, *out_len, h);
    std::snprintf(name_out, 64, "%s", base32_nopad(h, 32).c_str());
  }
  return CE_OK;
}
}  // namespace ce

extern "C" {

int ce_core_compact_ops_device(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                               uint64_t blob_len, const uint8_t* actors, uint32_t m,
                               const uint32_t* d_file_actor, const uint64_t* d_file_version,
                               const uint8_t* nonce, ce_buf* file, char name_out[64]) {
  if (!c || !file || (n && (!d_blob || !d_offs || !actors || !d_file_actor || !d_file_version)))
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  const uint8_t* p = nullptr;
  size_t len = 0;
  int rc = compact_ops_device_impl(c, d_blob, d_offs, n, blob_len, actors, m, d_file_actor, d_file_version,
                                   nonce, &p, &len, name_out);
  if (rc) return rc;
  file->data = (uint8_t*)malloc(len ? len : 1);
  std::memcpy(file->data, p, len);
  file->len = len;
  return CE_OK;
}

int ce_core_compact_ops_device_into(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                                    uint64_t blob_len, const uint8_t* actors, uint32_t m,
                                    const uint32_t* d_file_actor, const uint64_t* d_file_version,
                                    const uint8_t* nonce, uint8_t* dst, size_t cap, size_t* len,
                                    char name_out[64]) {
  if (!c || !len || (cap && !dst) || (n && (!d_blob || !d_offs || !actors || !d_file_actor || !d_file_version)))
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  c->sink = dst;
  c->sink_cap = cap;
  const uint8_t* p = nullptr;
  size_t l = 0;
  int rc = compact_ops_device_impl(c, d_blob, d_offs, n, blob_len, actors, m, d_file_actor, d_file_version,
                                   nonce, &p, &l, name_out);
  c->sink = nullptr;
  c->sink_cap = 0;
  if (rc) return rc;
  *len = l;
  if (p != dst) {
    if (cap < l) return c->ctx->fail(CE_ERR_INVALID_ARG, "compact_ops_device_into: buffer too small");
    std::memcpy(dst, p, l);
  }
  return CE_OK;
}

int ce_core_compact_ops_iov(ce_core* c, const uint8_t* const* files, const size_t* lens, uint32_t n,
                            const uint8_t* actors, uint32_t m, const uint32_t* file_actor,
                            const uint64_t* file_version, const uint8_t* nonce, ce_buf* file,
                            char name_out[64]) {
  if (!c || !file || (n && (!files || !lens || !actors || !file_actor || !file_version)))
    return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  ce_ctx* ctx = c->ctx;
  std::vector<uint64_t> offs;
  iov_offsets(lens, n, &offs);
  hipError_t e;
  if ((e = c->d_meta.reserve(n * 12ull + 64))) return ctx->hip_fail(e, "meta");
  if (n) {
    int rc = stage_host_batch(ctx, files, offs.data(), n);
    if (rc) return rc;
    uint8_t* mb = c->d_meta.as<uint8_t>();
    if ((e = hipMemcpyAsync(mb, file_version, n * 8ull, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(mb + 8ull * n, file_actor, n * 4ull, hipMemcpyHostToDevice, ctx->stream)))
      return ctx->hip_fail(e, "meta upload");
  }
  const uint8_t* mb = c->d_meta.as<uint8_t>();
  return ce_core_compact_ops_device(c, ctx->blob.as<uint8_t>(), ctx->offs.as<uint64_t>(), n, offs[n],
                                    actors, m, reinterpret_cast<const uint32_t*>(mb + 8ull * n),
                                    reinterpret_cast<const uint64_t*>(mb), nonce, file, name_out);
}

int ce_core_ingest_states(ce_core* c, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                          int32_t* status) {
  if (!c || (n && (!blob || !offs))) return CE_ERR_INVALID_ARG;
  HostPhase hp("ingest_states (all)");
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  return ingest_states_host(c, blob, offs, n, status);
}

int ce_core_ingest_states_iov(ce_core* c, const uint8_t* const* files, const size_t* lens, uint32_t n,
                              int32_t* status) {
  if (!c || (n && (!files || !lens))) return CE_ERR_INVALID_ARG;
  HostPhase hp("ingest_states (all)");
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  std::vector<uint64_t> offs(n + 1, 0);
  for (uint32_t i = 0; i < n; i++) offs[i + 1] = offs[i] + lens[i];
  return ingest_states_host(c, nullptr, offs.data(), n, status, files);
}

int ce_core_ingest_states_device(ce_core* c, const uint8_t* d_blob, const uint64_t* d_offs, uint32_t n,
                                 uint64_t blob_len, int32_t* status) {
  if (!c || (n && (!d_blob || !d_offs))) return CE_ERR_INVALID_ARG;
  HostPhase hp("ingest_states_device (all)");
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  return ingest_states_dev(c, d_blob, d_offs, n, blob_len, status);
}

int ce_core_read_remote(ce_core* c) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  return read_remote(c);
}

int ce_core_compact_to_buffer(ce_core* c, const uint8_t* nonce, ce_buf* file, char name_out[64]) {
  if (!c || !file) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  std::vector<uint8_t>& f = c->file_buf;
  int rc = compact_bytes(c, nonce, &f);
  if (rc) return rc;
  if (name_out) {
    HostPhase hp("sha3 name");
    uint8_t h[32];
    sha3_256(f.data(), f.size(), h);
    std::snprintf(name_out, 64, "%s", base32_nopad(h, 32).c_str());
  }
  file->data = (uint8_t*)malloc(f.size() ? f.size() : 1);
  std::memcpy(file->data, f.data(), f.size());
  file->len = f.size();
  return CE_OK;
}

int ce_core_compact_into(ce_core* c, const uint8_t* nonce, uint8_t* dst, size_t cap, size_t* len,
                         char name_out[64]) {
  if (!c || !len || (cap && !dst)) return CE_ERR_INVALID_ARG;
  HostPhase hw("compact_into");
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  std::vector<uint8_t>& f = c->file_buf;
  c->sink = dst;
  c->sink_cap = cap;
  c->sink_len = 0;
  int rc = compact_bytes(c, nonce, &f);
  c->sink = nullptr;
  c->sink_cap = 0;
  if (rc) return rc;
  if (c->sink_len) {
    *len = c->sink_len;
  } else {
    *len = f.size();
    if (cap < f.size()) return c->ctx->fail(CE_ERR_INVALID_ARG, "compact_into: buffer too small");
    std::memcpy(dst, f.data(), f.size());
  }
  if (name_out) {
    HostPhase hp("sha3 name");
    uint8_t h[32];
    sha3_256(dst, *len, h);
    std::snprintf(name_out, 64, "%s", base32_nopad(h, 32).c_str());
  }
  return CE_OK;
}

int ce_core_compact_into_async(ce_core* c, const uint8_t* nonce, uint8_t* dst, size_t cap, size_t* len,
                               uint64_t* ticket) {
  if (!c || !len || !ticket || (cap && !dst)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  c->sink_async = true;
  c->sink_ticket = 0;
  const int rc = ce_core_compact_into(c, nonce, dst, cap, len, nullptr);
  c->sink_async = false;
  *ticket = rc == CE_OK ? c->sink_ticket : 0;   // 0: already complete (small or host-written file)
  c->sink_ticket = 0;
  return rc;
}

int ce_core_compact_wait(ce_core* c, uint64_t ticket, uint64_t* len) {
  if (!c) return CE_ERR_INVALID_ARG;
  if (ticket == 0) return CE_OK;
  hipEvent_t ev = nullptr;
  hsa_signal_t sig{0};
  bool dma = false;
  uint32_t slot;
  {
    std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
    if (ticket > c->copy_next) return CE_ERR_INVALID_ARG;
    slot = (uint32_t)(ticket % ce_core::kAsyncSlots);
    if (c->copy_slot_ticket[slot] != ticket)  // the slot was reused (synchronised then): its length is gone
      return len ? c->ctx->fail(CE_ERR_INVALID_ARG, "compact ticket expired") : CE_OK;
    if (c->pend && c->pend_slot == slot) {  // its download not enqueued yet: wait for the seal, enqueue
      const int rk = ds_async_kick(c, true);
      if (rk) return rk;
    }
    ev = c->copy_ev[slot];
    dma = c->copy_dma[slot];
    sig = c->copy_sig[slot];
  }
  // outside the context lock: other calls on this core may proceed meanwhile (the event and the
  // signal stay alive until the core is closed)
  if (dma) {
    ce::dma_wait(sig);
  } else {
    const hipError_t e = hipEventSynchronize(ev);
    if (e) return c->ctx->hip_fail(e, "compact wait");
  }
  const uint64_t n = c->copy_len.as<volatile uint64_t>()[slot];
  if (n == ~1ull) return c->ctx->fail(CE_ERR_DEVICE, "serializer overran its bound");
  if (n == ~0ull) return c->ctx->fail(CE_ERR_INVALID_ARG, "compact_into_async: buffer too small");
  if (len) *len = n;
  return CE_OK;
}

int ce_core_compact(ce_core* c, char name_out[64]) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (!c->storage) return c->ctx->fail(CE_ERR_INVALID_ARG, "core opened without storage");
  int rc = read_remote(c);
  if (rc) return rc;
  std::vector<uint8_t> f;
  if ((rc = compact_bytes(c, nullptr, &f))) return rc;
  const std::vector<std::string> states_to_remove(c->read_states.begin(), c->read_states.end());
  std::vector<std::pair<Uuid, uint64_t>> ops_to_remove;  // (actor, counter - 1) (lib.rs:340-345)
  for (uint32_t s = 0; s < c->cap; s++)
    if (c->h_table[s].used && c->nov[s]) ops_to_remove.push_back({c->slot_actor[s], c->nov[s] - 1});
  std::string name;
  if ((rc = storage_store_content(c->storage, "states", f.data(), f.size(), &name)))
    return c->ctx->fail(rc, "failed writing state file");
  for (auto& s : states_to_remove)
    if ((rc = storage_remove_state(c->storage, s))) return c->ctx->fail(rc, "failed removing state file");
  for (auto& o : ops_to_remove)
    if ((rc = storage_remove_op(c->storage, o.first, o.second))) return c->ctx->fail(rc, "failed removing ops file");
  for (auto& s : states_to_remove) c->read_states.erase(s);
  c->read_states.insert(name);
  if (name_out) std::snprintf(name_out, 64, "%s", name.c_str());
  return CE_OK;
}

int ce_core_apply_ops(ce_core* c, const uint8_t* ops, size_t len) {
  if (!c || (len && !ops)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (!c->has_key) return c->ctx->fail(CE_ERR_NO_KEY, "no latest key");
  Dots dots;
  const bool ds = is_dotset_kind(c->kind);
  if (ds) {
    int rc = ds_check_ops(c, ops, len);
    if (rc) return rc;
  } else if (!read_dots(ops, len, &dots)) {
    return c->ctx->fail(CE_ERR_DECODE, "ops are not a Vec<Dot<Uuid>>");
  }
  // clear_text = VersionBytes(current_data_version, msgpack(ops)).serialize() (lib.rs:670-671)
  std::vector<uint8_t> clear(c->current_data_version.begin(), c->current_data_version.end());
  clear.insert(clear.end(), ops, ops + len);
  std::vector<uint8_t> file;
  int rc = seal_one(c->ctx, key_of(c), kCoreVersion, nullptr, clear.data(), clear.size(), &file);
  if (rc) return rc;
  uint32_t s;
  if ((rc = insert_actor(c, c->local_actor, &s))) return rc;
  const uint64_t version = c->nov[s];  // next_op_versions.get(actor) (lib.rs:703)
  if (c->storage && (rc = storage_store_op(c->storage, c->local_actor, version, file.data(), file.size())))
    return c->ctx->fail(rc, "failed writing ops file");
  // state.apply(op) for op in ops (lib.rs:710-712)
  if ((rc = ds ? ds_apply_local_ops(c, ops, len) : merge_dots_host(c, dots))) return rc;
  // the apply may have grown the table (new Dot actors), which moves every slot: look it up again
  s = c->slot_of.at(c->local_actor);
  c->nov[s] = version + 1;                         // next_op_versions.inc(actor) (lib.rs:714-715)
  return table_upload(c);
}

// n successive Core::apply_ops calls (lib.rs:666-722) as one batch: every clear text
// VersionBytes(current_data_version, ops_i) sealed by one GPU launch under the latest key, file i
// stored as ops/<local actor>/<next_op_versions.get(actor) + i>, the ops applied in order and
// next_op_versions bumped by n.  Every ops blob is decoded before anything is sealed or written.
int ce_core_apply_ops_batch(ce_core* c, const uint8_t* ops, const uint64_t* offs, uint32_t n,
                            const uint8_t* nonces, ce_buf* files, ce_buf* file_offs) {
  if (!c || (n && (!ops || !offs))) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  ce_ctx* ctx = c->ctx;
  if (!c->has_key) return ctx->fail(CE_ERR_NO_KEY, "no latest key");
  const bool ds = is_dotset_kind(c->kind);
  std::vector<Dots> dots(ds ? 0 : n);
  for (uint32_t i = 0; i < n; i++) {
    const uint8_t* p = ops + offs[i];
    const size_t l = offs[i + 1] - offs[i];
    if (ds) {
      int rc = ds_check_ops(c, p, l);
      if (rc) return rc;
    } else if (!read_dots(p, l, &dots[i])) {
      return ctx->fail(CE_ERR_DECODE, "ops are not a Vec<Dot<Uuid>>");
    }
  }
  // clear text i = current_data_version || ops_i (lib.rs:670-671); file i = CURRENT_VERSION ||
  // Cryptor::encrypt(clear_i) (lib.rs:682-695)
  std::vector<uint64_t> coffs(n + 1), foffs(n + 1);
  coffs[0] = foffs[0] = 0;
  for (uint32_t i = 0; i < n; i++) {
    coffs[i + 1] = coffs[i] + 16 + (offs[i + 1] - offs[i]);
    foffs[i + 1] = foffs[i] + 16 + sealed_len(16 + (offs[i + 1] - offs[i]));
  }
  std::vector<uint8_t> clear(coffs[n]);
  for (uint32_t i = 0; i < n; i++) {
    std::memcpy(clear.data() + coffs[i], c->current_data_version.data(), 16);
    std::memcpy(clear.data() + coffs[i] + 16, ops + offs[i], offs[i + 1] - offs[i]);
  }
  std::vector<uint8_t> nb;
  if (!nonces) {
    nb.resize(24ull * n + 1);
    os_random(nb.data(), 24ull * n);
    nonces = nb.data();
  }
  std::vector<uint8_t> out(foffs[n]);
  if (n) {
    hipError_t e;
    if ((e = ctx->blob.reserve(coffs[n] + 64)) || (e = ctx->offs.reserve((n + 1) * 8ull)) ||
        (e = ctx->out_offs.reserve((n + 1) * 8ull)) || (e = ctx->nonces.reserve(24ull * n)) ||
        (e = ctx->out.reserve(foffs[n] + 64)) || (e = ctx->outer_ver.reserve(64)))
      return ctx->hip_fail(e, "apply_ops_batch reserve");
    if ((e = hipMemcpyAsync(ctx->blob.p, clear.data(), coffs[n], hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->offs.p, coffs.data(), (n + 1) * 8ull, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->out_offs.p, foffs.data(), (n + 1) * 8ull, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->nonces.p, nonces, 24ull * n, hipMemcpyHostToDevice, ctx->stream)) ||
        (e = hipMemcpyAsync(ctx->outer_ver.p, kCoreVersion, 16, hipMemcpyHostToDevice, ctx->stream)))
      return ctx->hip_fail(e, "apply_ops_batch upload");
    int rc = device_seal(ctx, ctx->blob.as<uint8_t>(), ctx->offs.as<uint64_t>(), n, coffs[n],
                         ctx->outer_ver.as<uint8_t>(), ctx->nonces.as<uint8_t>(), ctx->out.as<uint8_t>(),
                         ctx->out_offs.as<uint64_t>(), key_of(c));
    if (rc) return rc;
    if ((e = hipMemcpyAsync(out.data(), ctx->out.p, foffs[n], hipMemcpyDeviceToHost, ctx->stream)) ||
        (e = stream_wait(ctx->stream)))
      return ctx->hip_fail(e, "apply_ops_batch download");
  }
  uint32_t s;
  int rc = insert_actor(c, c->local_actor, &s);
  if (rc) return rc;
  const uint64_t v0 = c->nov[s];  // next_op_versions.get(actor) (lib.rs:703)
  for (uint32_t i = 0; i < n; i++) {
    if (c->storage && (rc = storage_store_op(c->storage, c->local_actor, v0 + i, out.data() + foffs[i],
                                             foffs[i + 1] - foffs[i])))
      return ctx->fail(rc, "failed writing ops file");
    // state.apply(op) for op in ops (lib.rs:710-712), then next_op_versions.inc (lib.rs:714-715)
    if ((rc = ds ? ds_apply_local_ops(c, ops + offs[i], offs[i + 1] - offs[i]) : merge_dots_host(c, dots[i])))
      return rc;
    s = c->slot_of.at(c->local_actor);  // a growth inside the apply moved the local actor's slot
    c->nov[s] = v0 + i + 1;
  }
  if (files) {
    files->data = (uint8_t*)malloc(out.size() ? out.size() : 1);
    std::memcpy(files->data, out.data(), out.size());
    files->len = out.size();
  }
  if (file_offs) {
    file_offs->data = (uint8_t*)malloc((n + 1) * 8ull);
    std::memcpy(file_offs->data, foffs.data(), (n + 1) * 8ull);
    file_offs->len = (n + 1) * 8ull;
  }
  return table_upload(c);
}

int ce_core_reset(ce_core* c) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  std::fill(c->nov.begin(), c->nov.end(), 0);
  c->read_states.clear();
  if (is_dotset_kind(c->kind)) return ds_reset(c);  // (the dense state array is the VClock kinds')
  hipError_t e = hipMemsetAsync(c->d_state.p, 0, c->cap * 8ull, c->ctx->stream);
  if (e) return c->ctx->hip_fail(e, "reset");
  return CE_OK;
}

int ce_core_settle(ce_core* c) {
  if (!c) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  if (is_dotset_kind(c->kind)) return ds_settle(c);
  hipError_t e = hipStreamSynchronize(c->ctx->stream);
  if (e) return c->ctx->hip_fail(e, "settle");
  return CE_OK;
}

int ce_core_register_actors(ce_core* c, const uint8_t* actors, uint32_t m) {
  if (!c || (m && !actors)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  if (c->registered != c->size) return CE_ERR_INVALID_ARG;
  while ((c->size + m) * kTableLoadInv > c->cap) {
    int rc = table_grow(c);
    if (rc) return rc;
  }
  for (uint32_t i = 0; i < m; i++) {
    Uuid u;
    std::memcpy(u.data(), actors + 16ull * i, 16);
    uint32_t s;
    int rc = insert_actor(c, u, &s);
    if (rc) return rc;
  }
  c->registered = c->size;
  return table_upload(c);
}

uint32_t ce_core_dense_capacity(ce_core* c) { return c ? c->cap : 0; }

uint64_t ce_core_path_count(ce_core* c, const char* path) {
  if (!c || !path) return 0;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  auto it = c->path_counts.find(path);
  return it == c->path_counts.end() ? 0 : it->second;
}

int ce_core_dense_ready(ce_core* c) {
  if (!c || is_dotset_kind(c->kind)) return 0;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  return c->registered == c->size ? 1 : 0;
}

int ce_core_export_dense(ce_core* c, uint64_t* d_state, uint64_t* d_nov) {
  if (!c || !d_state || !d_nov || is_dotset_kind(c->kind)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  if (c->registered != c->size) return c->ctx->fail(CE_ERR_INVALID_ARG, "actors outside the registered set");
  hipError_t e;
  if ((e = hipMemcpyAsync(d_state, c->d_state.p, c->cap * 8ull, hipMemcpyDeviceToDevice, c->ctx->stream)) ||
      (e = hipMemcpyAsync(d_nov, c->nov.data(), c->cap * 8ull, hipMemcpyHostToDevice, c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "export");
  return CE_OK;
}

int ce_core_import_dense(ce_core* c, const uint64_t* d_state, const uint64_t* d_nov) {
  if (!c || !d_state || !d_nov || is_dotset_kind(c->kind)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  if (c->registered != c->size) return c->ctx->fail(CE_ERR_INVALID_ARG, "actors outside the registered set");
  std::vector<uint64_t> nv(c->cap);
  hipError_t e;
  if ((e = launch_merge_max(c->ctx->stream, c->d_state.as<unsigned long long>(),
                            reinterpret_cast<const unsigned long long*>(d_state), c->cap)) ||
      (e = hipMemcpyAsync(nv.data(), d_nov, c->cap * 8ull, hipMemcpyDeviceToHost, c->ctx->stream)) ||
      (e = stream_wait(c->ctx->stream)))
    return c->ctx->hip_fail(e, "import");
  for (uint32_t s = 0; s < c->cap; s++) c->nov[s] = std::max(c->nov[s], nv[s]);
  return CE_OK;
}

int ce_core_merge_state(ce_core* c, const uint8_t* sw, size_t len) {
  if (!c || (len && !sw)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (is_dotset_kind(c->kind)) {
    std::vector<std::pair<const uint8_t*, size_t>> sws{{sw, len}};
    int32_t st = CE_OK;
    return ds_merge_states(c, sws, &st, nullptr);
  }
  Dots nov, state;
  if (!read_state_wrapper(sw, len, c->kind, &nov, &state))
    return c->ctx->fail(CE_ERR_DECODE, "not a StateWrapper");
  int rc = merge_dots_host(c, state);  // state.merge(sw.state) (lib.rs:460)
  if (rc) return rc;
  for (auto& d : nov) {                // next_op_versions.merge(..) (lib.rs:461-463)
    uint32_t s;
    if ((rc = insert_actor(c, d.first, &s))) return rc;
    c->nov[s] = std::max(c->nov[s], d.second);
  }
  return table_upload(c);
}

// ce_core_state_bytes into device memory: Orswot through the device writer (the 35 MB C3
// partial never crosses PCIe); the other kinds' states are small and serialized on the host.
int ce_core_state_bytes_device(ce_core* c, uint8_t* d_dst, uint64_t cap, uint64_t* len) {
  if (!c || !len || (cap && !d_dst)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (c->kind == CE_STATE_ORSWOT && !c->host_compact) return ds_state_bytes_device(c, c->ctx, d_dst, cap, len);
  std::vector<uint8_t>& b = c->ser_buf;
  int rc = serialize_state(c, &b);
  if (rc) return rc;
  *len = b.size();
  if (b.size() > cap) return c->ctx->fail(CE_ERR_INVALID_ARG, "device buffer too small for the state");
  hipError_t e;
  if (!b.empty() && ((e = hipMemcpyAsync(d_dst, b.data(), b.size(), hipMemcpyHostToDevice, c->ctx->stream)) ||
                     (e = stream_wait(c->ctx->stream))))
    return c->ctx->hip_fail(e, "state bytes");
  return CE_OK;
}

// ce_core_merge_state over a StateWrapper resident in HBM: Orswot through the device state
// reader (ds_merge_states_device: only the head -- next_op_versions and the clock -- and the
// deferred tail come to the host); the other kinds download it (small) and merge on the host.
int ce_core_merge_state_device(ce_core* c, const uint8_t* d_sw, uint64_t len) {
  if (!c || (len && !d_sw)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (c->kind == CE_STATE_ORSWOT && !getenv("CE_HOST_STATES")) {
    int32_t st = CE_OK;
    return ds_merge_states_device(c, d_sw, std::vector<uint64_t>{0}, std::vector<uint64_t>{len}, &st, nullptr);
  }
  std::vector<uint8_t> h(len);
  hipError_t e;
  if (len && ((e = hipMemcpyAsync(h.data(), d_sw, len, hipMemcpyDeviceToHost, c->ctx->stream)) ||
              (e = stream_wait(c->ctx->stream))))
    return c->ctx->hip_fail(e, "merge state");
  return ce_core_merge_state(c, h.data(), len);
}

int ce_core_export_columns_device(ce_core* c, uint8_t* d_dst, uint64_t cap, uint64_t* len) {
  if (!c || !len || (cap && !d_dst)) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  *len = 0;
  if (c->kind != CE_STATE_ORSWOT || c->host_compact)
    return c->ctx->fail(CE_ERR_INVALID_ARG, "no column form for this state kind: use the state bytes");
  return ds_export_columns_device(c, d_dst, cap, len);
}

int ce_core_merge_columns_device(ce_core* c, const uint8_t* const* d_parts, const uint64_t* lens, uint32_t k) {
  if (!c || (k && (!d_parts || !lens))) return CE_ERR_INVALID_ARG;
  std::lock_guard<std::recursive_mutex> g(c->ctx->mu);
  (void)hipSetDevice(c->ctx->device);
  if (c->kind != CE_STATE_ORSWOT || c->host_compact)
    return c->ctx->fail(CE_ERR_INVALID_ARG, "no column form for this state kind: use the state bytes");
  return ds_merge_columns_device(c, d_parts, lens, k);
}

void* ce_host_alloc(size_t bytes) {
  void* p = nullptr;
  return hipHostMalloc(&p, bytes ? bytes : 1, 0) == hipSuccess ? p : nullptr;
}

void ce_host_free(void* p) {
  if (p) (void)hipHostFree(p);
}

}  // extern "C"
