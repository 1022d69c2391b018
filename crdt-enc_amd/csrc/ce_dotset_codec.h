// ce_dotset_codec.h -- rmp-serde `from_slice` decoding of the dot-set op vectors on the fold
// path, shared by the device decode kernel (ce_dotset.hip, one lane per file) and the host
// (state files, local ops): Vec<orswot::Op<u64, Uuid>> and Vec<mvreg::Op<u64, Uuid>>
// (crdt-enc/src/lib.rs:507 `rmp_serde::from_slice` of `Vec<S::Op>`).
//
// Wire forms accepted (rmp-serde 1.x; enum form *parity unpinned*):
//   enum        map of exactly one entry {variant: body}, variant = name str or index uint
//   struct      map keyed by field name / index (any order, unknown keys skipped, duplicates
//               rejected, all fields required) or array of exactly the field count
//   VClock      struct {dots: map<Uuid, u64>}
//   Uuid        bin16 (or non-UTF-8 str16, see rd_uuid)
//   u64         any non-negative msgpack integer
// A VClock whose actors are not strictly ascending (BTreeMap order; a repeated actor keeps the
// later value) or nesting deeper than kMaxDepth is reported as -1 ("host parse"): the host
// decoder handles it with the same rules.
#pragma once
#include "ce_common.h"

namespace ce {

// result codes of the parsers: 1 ok, 0 decode error (CE_ERR_DECODE), -1 host parse
enum { kDsErr = 0, kDsOk = 1, kDsHost = -1 };

// read an enum header: map(1) then the variant identifier; returns variant index, -2 error
template <int NV, typename R>
CE_HD int ds_variant(R& r, const char* const (&names)[NV]) {
  uint64_t cnt;
  if (r.i >= r.n || !is_map_marker(rb(r, r.i))) return -2;
  if (!rd_map_hdr(r, &cnt) || cnt != 1) return -2;
  const int v = rd_field<NV>(r, names);
  return (v < 0 || v >= NV) ? -2 : v;
}

// Vec<u64>: calls sink.member(m) for each element
template <typename R, typename F>
CE_HD int ds_members(R& r, F&& member) {
  uint64_t cnt, m;
  if (r.i >= r.n || !is_array_marker(rb(r, r.i))) return kDsErr;
  if (!rd_array_hdr(r, &cnt) || cnt > r.n - r.i) return kDsErr;
  for (uint64_t k = 0; k < cnt; k++) {
    if (!rd_u64(r, &m)) return kDsErr;
    member(m);
  }
  return kDsOk;
}

// VClock {dots: map<Uuid, u64>}: calls dot(actor_off, counter) per entry.
template <typename R, typename F>
CE_HD int ds_vclock(R& r, F&& dot) {
  static constexpr const char* kF[1] = {"dots"};
  if (r.i >= r.n) return kDsErr;
  uint64_t cnt;
  const uint8_t m0 = rb(r, r.i);
  bool have = false;
  auto dots = [&](R& q) -> int {
    uint64_t n, off, c, prev = 0;
    if (!rd_map_hdr(q, &n) || n > q.n - q.i) return kDsErr;
    for (uint64_t k = 0; k < n; k++) {
      if (!rd_uuid(q, &off) || !rd_u64(q, &c)) return kDsErr;
      // BTreeMap serializes keys strictly ascending; any other order may repeat an actor
      // (the later value wins on insert) -> host decoder
      if (k) {
        int cmp = 0;
        for (int b = 0; b < 16 && cmp == 0; b++)
          cmp = (int)q.p[off + b] - (int)q.p[prev + b];  // direct: two keys apart
        if (cmp <= 0) return kDsHost;
      }
      prev = off;
      dot(off, c);
    }
    return kDsOk;
  };
  if (is_array_marker(m0)) {
    if (!rd_array_hdr(r, &cnt) || cnt != 1) return kDsErr;
    return dots(r);
  }
  if (!rd_map_hdr(r, &cnt)) return kDsErr;
  for (uint64_t k = 0; k < cnt; k++) {
    const int f = rd_field<1>(r, kF);
    if (f < 0) return kDsErr;
    if (f == 1) {
      const int s = rd_skip(r);
      if (s <= 0) return s == 0 ? kDsErr : kDsHost;
      continue;
    }
    if (have) return kDsErr;
    have = true;
    const int s = dots(r);
    if (s != kDsOk) return s;
  }
  return have ? kDsOk : kDsErr;
}

// Struct body with two fields, each parsed by fn(field_index, rd) -> kDs*.
template <typename R, typename F>
CE_HD int ds_struct2(R& r, const char* const (&names)[2], F&& fn) {
  if (r.i >= r.n) return kDsErr;
  uint64_t cnt;
  if (is_array_marker(rb(r, r.i))) {
    if (!rd_array_hdr(r, &cnt) || cnt != 2) return kDsErr;
    for (int f = 0; f < 2; f++) {
      const int s = fn(f, r);
      if (s != kDsOk) return s;
    }
    return kDsOk;
  }
  if (!rd_map_hdr(r, &cnt)) return kDsErr;
  unsigned seen = 0;
  for (uint64_t k = 0; k < cnt; k++) {
    const int f = rd_field<2>(r, names);
    if (f < 0) return kDsErr;
    if (f == 2) {
      const int s = rd_skip(r);
      if (s <= 0) return s == 0 ? kDsErr : kDsHost;
      continue;
    }
    if (seen & (1u << f)) return kDsErr;
    seen |= 1u << f;
    const int s = fn(f, r);
    if (s != kDsOk) return s;
  }
  return seen == 3u ? kDsOk : kDsErr;
}

// Sink interface for Orswot ops (all calls of one op come between begin/end):
//   add_begin(); add_dot(actor_off, counter); add_member(m); add_end();
//   rm_begin();  rm_dot(actor_off, counter);  rm_member(m);  rm_end();
// Fields may come in any order (struct maps), so a sink must not assume dot-before-members.
// One orswot::Op at r.i (the element grammar of the Vec below).
template <typename R, typename S>
CE_HD int ds_orswot_op(R& r, S& sink) {
  static constexpr const char* kV[2] = {"Add", "Rm"};
  static constexpr const char* kAdd[2] = {"dot", "members"};
  static constexpr const char* kRm[2] = {"clock", "members"};
  const int v = ds_variant<2>(r, kV);
  if (v < 0) return kDsErr;
  int s;
  if (v == 0) {
    sink.add_begin();
    s = ds_struct2(r, kAdd, [&](int f, R& q) -> int {
      if (f == 1) return ds_members(q, [&](uint64_t m) { sink.add_member(m); });
      uint64_t aoff, c;
      const int d = parse_dot(q, &aoff, &c);
      if (d <= 0) return d == 0 ? kDsErr : kDsHost;
      sink.add_dot(aoff, c);
      return kDsOk;
    });
    if (s == kDsOk) sink.add_end();
  } else {
    sink.rm_begin();
    s = ds_struct2(r, kRm, [&](int f, R& q) -> int {
      if (f == 1) return ds_members(q, [&](uint64_t m) { sink.rm_member(m); });
      return ds_vclock(q, [&](uint64_t off, uint64_t c) { sink.rm_dot(off, c); });
    });
    if (s == kDsOk) sink.rm_end();
  }
  return s;
}

template <typename S, typename R = Rd>
CE_HD int ds_parse_orswot_ops(const uint8_t* p, uint64_t n, S& sink) {
  R r{p, n, 0};
  uint64_t cnt;
  if (r.n == 0 || !is_array_marker(rb(r, 0)) || !rd_array_hdr(r, &cnt) || cnt > r.n) return kDsErr;
  for (uint64_t k = 0; k < cnt; k++) {
    const int s = ds_orswot_op(r, sink);
    if (s != kDsOk) return s;
  }
  return kDsOk;  // rmp_serde::from_slice does not look past the value (as ce_fused's Vec<Dot>)
}

// Sink for MVReg ops: put_begin(); put_dot(actor_off, counter); put_val(v); put_end();
template <typename S, typename R = Rd>
CE_HD int ds_parse_mvreg_ops(const uint8_t* p, uint64_t n, S& sink) {
  static constexpr const char* kV[1] = {"Put"};
  static constexpr const char* kPut[2] = {"clock", "val"};
  R r{p, n, 0};
  uint64_t cnt;
  if (r.n == 0 || !is_array_marker(rb(r, 0)) || !rd_array_hdr(r, &cnt) || cnt > r.n) return kDsErr;
  for (uint64_t k = 0; k < cnt; k++) {
    const int v = ds_variant<1>(r, kV);
    if (v < 0) return kDsErr;
    sink.put_begin();
    const int s = ds_struct2(r, kPut, [&](int f, R& q) -> int {
      if (f == 0) return ds_vclock(q, [&](uint64_t off, uint64_t c) { sink.put_dot(off, c); });
      uint64_t val;
      if (!rd_u64(q, &val)) return kDsErr;
      sink.put_val(val);
      return kDsOk;
    });
    if (s != kDsOk) return s;
    sink.put_end();
  }
  return kDsOk;
}

}  // namespace ce
