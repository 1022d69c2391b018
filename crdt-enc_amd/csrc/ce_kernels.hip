// ce_kernels.hip -- gfx950 kernels of the compaction/ingest hot path.
//
//  k_open_setup     one lane per file: outer version (crdt-enc/src/lib.rs:501), envelope parse
//                   (crdt-enc-xchacha20poly1305/src/lib.rs:82-91), HChaCha20 subkey, Poly1305
//                   key (ChaCha20 block 0) and r^(2^k) k=0..6.
//  k_seal_setup     one lane per file: writes CURRENT_VERSION || msgpack header
//                   (xchacha lib.rs:59-67, crdt-enc/src/lib.rs:695), key schedule.
//  k_segments       one wavefront per 16 KiB segment: ChaCha20 keystream (one 64-byte block
//                   per lane, transposed through LDS), coalesced 16-byte pieces, Poly1305 as a
//                   64-way strided Horner in r^64 + a 6-level cross-lane tree in r^(2^k);
//                   single-segment files finalize in place (tag compare, scrub on failure).
//  k_finalize_multi one lane per multi-segment file: Horner over segment partials.
//  k_decode_dots    one wavefront per file: rmp-serde Vec<Dot<Uuid>> (crdt-enc/src/lib.rs:507)
//                   decoded 64 dots at a time by speculating on the canonical encoding, general
//                   grammar by lane 0 otherwise; dots of applied files max-folded
//                   (VClock::apply) into a dense batch state.
#include "ce_device.h"

namespace ce {

// ----------------------------------------------------------------------------------------
// setup kernels
// ----------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_open_setup(const uint8_t* __restrict__ blob,
                                                    const uint64_t* __restrict__ offs, uint32_t n,
                                                    int outer, DevKey key, int32_t key_status,
                                                    FileParams* __restrict__ params,
                                                    int32_t* __restrict__ status, SegScratch sc,
                                                    PolyAux* __restrict__ aux) {
  // parameters are staged in LDS, 128 B per lane per half (16-B columns XOR-swizzled by the
  // lane), and stored as the block's contiguous rows: a per-lane 256-B struct store touches 64
  // lines per instruction.  32 KiB keeps 5 workgroups per CU.  The PolyAux rows (when asked
  // for) go the same way as a third half.
  __shared__ uint4 stage[256 * 8];
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  const bool active = f < n;
  const uint64_t off = active ? offs[f] : 0;
  const uint64_t flen = active ? offs[f + 1] - off : 0;
  const uint8_t* enc = blob + off;
  uint64_t enc_len = flen;
  int32_t st = active ? CE_OK : CE_ERR_OUTER_LEN;
  if (active && outer) {
    // Storage: VersionBytes::deserialize (tokio lib.rs:241), then the core's
    // ensure_versions_phf(SUPPORTED_VERSIONS) (crdt-enc/src/lib.rs:501)
    if (flen < 16) st = CE_ERR_OUTER_LEN;
    else {
      // one (unaligned) 16-byte load against the version's little-endian words
      const uint4 v = *reinterpret_cast<const uint4*>(enc);
      auto le = [](int i) {
        return (uint32_t)kCoreVersion[4 * i] | ((uint32_t)kCoreVersion[4 * i + 1] << 8) |
               ((uint32_t)kCoreVersion[4 * i + 2] << 16) | ((uint32_t)kCoreVersion[4 * i + 3] << 24);
      };
      if (v.x != le(0) || v.y != le(1) || v.z != le(2) || v.w != le(3)) st = CE_ERR_OUTER_VERSION;
      enc += 16;
      enc_len -= 16;
    }
  }
  if (st == CE_OK) st = key_status;  // key version / length (xchacha lib.rs:74-78)
  Envelope e{};
  bool fast = false;
  uint32_t nw[6];  // nonce words (fast path: from the header registers)
  if (st == CE_OK && enc_len >= 67 + 16) {
    // canonical EncHandler::encrypt box with a bin16 EncBox (clear text ~190 B .. 64 KiB),
    // checked from registers: 92 c4 10 <box16> c5 EE EE 82 a5"nonce" c4 18 <24> a8"enc_data"
    // c5 LL LL <ct||tag>  (xchacha lib.rs:59-67)
    uint32_t w[17];
#pragma unroll
    for (int i = 0; i < 4; i++) {
      const uint4 v = *reinterpret_cast<const uint4*>(enc + 16 * i);
      w[4 * i] = v.x; w[4 * i + 1] = v.y; w[4 * i + 2] = v.z; w[4 * i + 3] = v.w;
    }
    w[16] = ld_le32(enc + 64);
    auto byte = [&](int i) -> uint32_t { return (w[i >> 2] >> (8 * (i & 3))) & 0xffu; };
    bool ok = byte(0) == 0x92 && byte(1) == 0xc4 && byte(2) == 0x10 && byte(19) == 0xc5 &&
              byte(22) == 0x82 && byte(23) == 0xa5 && byte(24) == 'n' && byte(25) == 'o' &&
              byte(26) == 'n' && byte(27) == 'c' && byte(28) == 'e' && byte(29) == 0xc4 &&
              byte(30) == 0x18 && byte(55) == 0xa8 && byte(56) == 'e' && byte(57) == 'n' &&
              byte(58) == 'c' && byte(59) == '_' && byte(60) == 'd' && byte(61) == 'a' &&
              byte(62) == 't' && byte(63) == 'a' && byte(64) == 0xc5;
#pragma unroll
    for (int i = 0; i < 16; i++) ok = ok && byte(3 + i) == kBoxVersion[i];
    const uint32_t eb = (byte(20) << 8) | byte(21);
    const uint32_t l2 = (byte(65) << 8) | byte(66);
    if (ok && eb == 45 + l2 && 22ull + eb <= enc_len && l2 >= 16) {
      e.nonce_off = 31; e.nonce_len = 24; e.enc_off = 67; e.enc_len = l2;
      fast = true;
#pragma unroll
      for (int k = 0; k < 6; k++) nw[k] = __builtin_amdgcn_alignbyte(w[8 + k], w[7 + k], 3);  // bytes 31..54
    }
  }
  if (st == CE_OK && !fast) st = parse_envelope(enc, enc_len, &e);
  FileParams P;
  P.status = st;
  P.len = 0;
  P.in_off = 0;
  P.out_off = (off + 15) & ~15ull;
  P.nseg = 0;
  P.extra_base = 0;
  if (st == CE_OK) {
    const uint64_t ct_off = (uint64_t)(enc - blob) + e.enc_off;
    P.in_off = ct_off;
    P.len = (uint32_t)(e.enc_len - 16);
    const uint4 t = *reinterpret_cast<const uint4*>(blob + ct_off + P.len);  // unaligned 16 B
    P.tag[0] = t.x; P.tag[1] = t.y; P.tag[2] = t.z; P.tag[3] = t.w;
    if (!fast) {
#pragma unroll
      for (int k = 0; k < 6; k++) nw[k] = ld_le32(enc + e.nonce_off + 4 * k);
    }
    key_schedule_w(key, nw, P);
    if (P.len > kSmallMax) sc.large_list[atomicAdd(&sc.counters[9], 1u)] = f;
  }
  reserve_segments(P, f, sc, st == CE_OK);  // the whole wave (long files are filled together)
  PolyAux X;
  if (aux) {  // block-uniform
    if (st == CE_OK) poly_aux(P, X);
    else X = PolyAux{};
  }
  {
    const uint4* pv = reinterpret_cast<const uint4*>(&P);
    const uint4* xv = reinterpret_cast<const uint4*>(&X);
    const uint32_t f0 = blockIdx.x * blockDim.x;
    const uint32_t nrow = min(n - f0, (uint32_t)blockDim.x);
    uint4* dstp = reinterpret_cast<uint4*>(params + f0);
    uint4* dsta = aux ? reinterpret_cast<uint4*>(aux + f0) : nullptr;
#pragma unroll
    for (int h = 0; h < 3; h++) {
      if (h == 2 && !aux) break;
      if (h) __syncthreads();
#pragma unroll
      for (int i = 0; i < 8; i++) stage[threadIdx.x * 8 + (i ^ (threadIdx.x & 7))] = h < 2 ? pv[8 * h + i] : xv[i];
      __syncthreads();
#pragma unroll
      for (int k = 0; k < 8; k++) {
        const uint32_t j = threadIdx.x + 256u * k;
        const uint32_t row = j >> 3, col = j & 7;
        if (row < nrow) {
          const uint4 v = stage[row * 8 + (col ^ (row & 7))];
          if (h < 2) dstp[row * 16 + 8 * h + col] = v;
          else dsta[row * 8 + col] = v;
        }
      }
    }
  }
  if (!active) return;
  status[f] = st;
  // counters once per wave (a batch under a wrong key fails every file: per-file atomics on
  // these words would serialise in L2); the lowest set lane holds the wave's lowest index
  const uint32_t lane = threadIdx.x & 63;
  const unsigned long long hp = __ballot(active && st == kStatusHostParse);
  const unsigned long long bad = __ballot(active && st != CE_OK && st != kStatusHostParse);
  if (hp && lane == (uint32_t)__builtin_ctzll(hp)) atomicAdd(&sc.counters[7], (uint32_t)__builtin_popcountll(hp));
  if (bad && lane == (uint32_t)__builtin_ctzll(bad)) {
    atomicAdd(&sc.counters[8], (uint32_t)__builtin_popcountll(bad));
    atomicMin(&sc.counters[5], f);
  }
}

__global__ __launch_bounds__(256) void k_seal_setup(const uint8_t* __restrict__ clear,
                                                    const uint64_t* __restrict__ offs, uint32_t n,
                                                    const uint8_t* __restrict__ outer_version,
                                                    const uint8_t* __restrict__ nonces,
                                                    uint8_t* __restrict__ out,
                                                    const uint64_t* __restrict__ out_offs,
                                                    DevKey key, FileParams* __restrict__ params,
                                                    SegScratch sc) {
  const uint32_t f = blockIdx.x * blockDim.x + threadIdx.x;
  const bool mine = f < n;
  FileParams P;
  P.len = 0;
  if (mine) {
    const uint64_t off = offs[f];
    const uint64_t len = offs[f + 1] - off;
    uint8_t* o = out + out_offs[f];
    uint64_t k = 0;
    if (outer_version) {
#pragma unroll
      for (int i = 0; i < 16; i++) o[i] = outer_version[i];
      k = 16;
    }
    const uint8_t* nonce = nonces + 24ull * f;
    uint8_t nb[24];
#pragma unroll
    for (int i = 0; i < 24; i++) nb[i] = nonce[i];
    // straight into the output (a local staging array was private scratch, read back byte by
    // byte: most of this kernel's ~14 us on a compaction's single file)
    const uint64_t h = put_envelope_header(o + k, len, nb);
    P.status = CE_OK;
    P.in_off = off;
    P.out_off = out_offs[f] + k + h;
    P.len = (uint32_t)len;
    key_schedule(key, nb, P);
  }
  reserve_segments(P, f, sc, mine);  // the whole wave (a long file's work items filled together)
  if (mine) params[f] = P;
}

// ----------------------------------------------------------------------------------------
// segment kernel: one wavefront per (file, 16 KiB segment)
// ----------------------------------------------------------------------------------------
static constexpr int kWavesPerBlock = 4;
static constexpr uint32_t kSegBytes = kSegBlocks * 16;

__device__ void decode_file(const DecodeArgs& a, uint32_t f, uint32_t lane);

// the 48-byte window at pt + p (unaligned global loads)
__device__ __forceinline__ void dot_window(const uint8_t* pt, uint32_t p, uint32_t (&w)[12]) {
  const uint4 A = *reinterpret_cast<const uint4*>(pt + p);
  const uint4 B = *reinterpret_cast<const uint4*>(pt + p + 16);
  const uint4 C = *reinterpret_cast<const uint4*>(pt + p + 32);
  w[0] = A.x; w[1] = A.y; w[2] = A.z; w[3] = A.w;
  w[4] = B.x; w[5] = B.y; w[6] = B.z; w[7] = B.w;
  w[8] = C.x; w[9] = C.y; w[10] = C.z; w[11] = C.w;
}

// slot of an actor through a one-entry per-lane cache (a file's Dots are mostly its writer's)
struct SlotCache {
  uint32_t c0 = 0, c1 = 0, c2 = 0, c3 = 0, slot = 0xffffffffu;
  __device__ __forceinline__ uint32_t get(const DecodeArgs& a, uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3) {
    if (slot != 0xffffffffu && k0 == c0 && k1 == c1 && k2 == c2 && k3 == c3) return slot;
    const uint32_t s = lookup_slot1(a.table, a.mask, a.nil_actor, k0, k1, k2, k3);
    if (s != 0xffffffffu) { c0 = k0; c1 = k1; c2 = k2; c3 = k3; slot = s; }
    return s;
  }
};

// C4's fused decode, part 1 (k_segments<false, true>, files of more than one segment): the
// canonical Dots lying wholly inside this segment's plaintext [S, E), decoded speculatively
// before the file's tag is known: segment 0 takes the Dot grid from the array header, a later
// segment from the first canonical Dot in its first 64 bytes.  Nothing is folded here; the
// record {first Dot offset | ~0, Dots, slot + 1 | 0 none | ~0 failed, Dot length},
// {max lo, max hi} is checked against the file's true grid by k_segdec_apply after the tag.
__device__ void seg_record(const DecodeArgs& a, const uint8_t* pt, uint32_t len, uint32_t S,
                           uint32_t E, uint32_t lane, uint4* rec) {
  uint32_t m = 0xffffffffu, L = 0, hcount = 0, hok = 0;
  if (S == 0) {
    // the file's header for k_segdec_apply too: supported data version, Dot count, and
    // whether the whole array fits the grid (crdt-enc/src/lib.rs:504-507)
    uint32_t hm = 0xffffffffu, hl = 0;
    if (lane == 0 && len >= 16) {
      const uint4 dv = *reinterpret_cast<const uint4*>(pt);
      bool found = false;
      for (uint32_t q = 0; q < a.n_supported; q++) {
        const uint4 sv = *reinterpret_cast<const uint4*>(a.supported + 16 * q);
        found |= dv.x == sv.x && dv.y == sv.y && dv.z == sv.z && dv.w == sv.w;
      }
      Rd r{pt + 16, len - 16, 0};
      uint64_t cnt = 0;
      if (rd_array_hdr(r, &cnt) && 16 + r.i + 34 <= E) {
        hm = 16 + (uint32_t)r.i;
        hl = dot_len_of_marker(pt[hm + 33]);
        if (hl == 0) hm = 0xffffffffu;
        hcount = cnt <= len ? (uint32_t)cnt : 0u;
        hok = found && hl != 0 && cnt <= len && (uint64_t)hm + cnt * hl <= len;
      }
    }
    m = bcast(hm);
    L = bcast(hl);
  } else {
    const uint32_t p = S + lane;
    uint32_t Ll = 0;
    bool v = false;
    if (p + 34 <= E) {
      Ll = dot_len_of_marker(pt[p + 33]);
      if (Ll != 0 && p + Ll <= E) {
        uint32_t w[12], k0, k1, k2, k3;
        unsigned long long ctr;
        dot_window(pt, p, w);
        v = canon_dot(w, Ll, k0, k1, k2, k3, ctr);
      }
    }
    const unsigned long long vm = __ballot(v);
    if (vm) {
      const uint32_t fl = (uint32_t)__builtin_ctzll(vm);
      m = S + fl;
      L = (uint32_t)__shfl((int)Ll, (int)fl);
    }
  }
  uint32_t nd = 0, myslot = 0xffffffffu;
  unsigned long long best = 0;
  bool fail = false;
  if (m != 0xffffffffu) {
    SlotCache cache;
    for (uint32_t base = m;;) {
      const uint32_t p = base + lane * L;
      const bool in = p + L <= E;
      uint32_t w[12], k0 = 0, k1 = 0, k2 = 0, k3 = 0;
      unsigned long long ctr = 0;
      dot_window(pt, in ? p : m, w);
      const bool valid = in && canon_dot(w, L, k0, k1, k2, k3, ctr);
      const unsigned long long vm = __ballot(valid);
      const uint32_t k = vm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~vm);
      if (lane < k) {
        const uint32_t sl = cache.get(a, k0, k1, k2, k3);
        if (sl == 0xffffffffu || (myslot != 0xffffffffu && sl != myslot)) fail = true;
        else {
          best = (myslot == 0xffffffffu || ctr > best) ? ctr : best;
          myslot = sl;
        }
      }
      nd += k;
      base += k * L;
      if (k < 64) break;
    }
  }
  uint32_t mx = myslot == 0xffffffffu ? 0u : myslot + 1;
  uint32_t mn = myslot == 0xffffffffu ? 0xffffffffu : myslot + 1;
  unsigned long long bm = best;
#pragma unroll
  for (int d = 32; d >= 1; d >>= 1) {
    const uint32_t omx = (uint32_t)__shfl_xor((int)mx, d), omn = (uint32_t)__shfl_xor((int)mn, d);
    const unsigned long long ob = __shfl_xor(bm, d);
    mx = omx > mx ? omx : mx;
    mn = omn < mn ? omn : mn;
    bm = ob > bm ? ob : bm;
  }
  const bool wfail = __ballot(fail) != 0 || (mx != 0 && mn != mx);
  if (lane == 0) {
    rec[0] = make_uint4(m, nd, wfail ? 0xffffffffu : mx, L);
    rec[1] = make_uint4((uint32_t)bm, (uint32_t)(bm >> 32), hcount, hok);
  }
}

// DEC (open only): decode during the segment pass -- a one-segment file is decoded and folded
// by its own wave once its tag verifies (decode_file, the plaintext just written is L2-hot); a
// longer file's segments leave seg_record records (rec, indexed like the Poly1305 partials)
template <bool SEAL, bool DEC>
__global__ __launch_bounds__(256) void k_segments(const uint8_t* __restrict__ in,
                                                  uint8_t* __restrict__ out,
                                                  const FileParams* __restrict__ params, uint32_t n,
                                                  int32_t* __restrict__ status, SegScratch sc,
                                                  int skip_small, DecodeArgs da, uint4* rec) {
  __shared__ __attribute__((aligned(16))) uint8_t lds[kWavesPerBlock * 64 * kKsStride];
  // the segment's Poly1305 multipliers r^64 .. r^256 (4 x MulR, wave-uniform) live in LDS and are
  // read back (broadcast) right where each product needs them: held in registers across the
  // page loop they cost 36 VGPRs, and the wave count per SIMD with them
  __shared__ __attribute__((aligned(16))) uint32_t mul_lds[kWavesPerBlock][36];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wib = threadIdx.x >> 6;
  uint8_t* ks = lds + wib * 64 * kKsStride;
  uint32_t* ml = mul_lds[wib];
  // skip_small: the first-segment work comes from the large-file list built by the setup
  const uint32_t nfirst = skip_small ? *((volatile uint32_t*)&sc.counters[9]) : n;
  const uint32_t total = nfirst + *((volatile uint32_t*)&sc.counters[0]);
  const uint32_t stride = gridDim.x * kWavesPerBlock;

  for (uint32_t w = bcast(blockIdx.x * kWavesPerBlock + wib); w < total; w += stride) {
    uint32_t f, j;
    if (w < nfirst) { f = skip_small ? bcast(sc.large_list[w]) : w; j = 0; }
    else { const uint2 e = sc.extra_list[w - nfirst]; f = bcast(e.x); j = bcast(e.y); }
    const FileParams* Pp = params + f;
    if (Pp->status != CE_OK) continue;  // setup status (never rewritten: read-only here)
    const uint32_t len = Pp->len;
    if (skip_small && len <= kSmallMax) continue;  // k_open_fold_small handles these
    const uint32_t nseg = Pp->nseg;
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = Pp->subkey[i];
    const uint32_t n2a = Pp->n2[0], n2b = Pp->n2[1];
    const L5 R = load_l5(Pp->rpow[6]);
    const uint8_t* src = in + Pp->in_off;
    uint8_t* dst = out + Pp->out_off;

    const uint32_t nblk_ct = (len + 15) >> 4;
    const uint32_t nblk = nblk_ct + 1;
    const uint32_t SB = SEAL ? sc.seg_blocks : kSegBlocks;  // (the open path keeps its constant)
    const uint32_t b_lo = j * SB;
    const uint32_t b_hi = min(nblk, b_lo + SB);
    const uint32_t nb = b_hi - b_lo;
    const uint32_t rows = (nb + 63) >> 6;

    L5 acc = {{0, 0, 0, 0, 0}};
    // A page whose 4 pieces are whole ciphertext pieces in every lane folds them as four products
    // into one set of column sums, acc R^4 + m0 R^3 + m1 R^2 + m2 R + m3 (R = r^64), reduced
    // once -- instead of four Horner mulmods.  Only the file's last page takes the Horner steps.
    {
      const L5 R2 = mulmod(R, R), R3 = mulmod(R2, R);
      const MulR Ms[4] = {mul_r(R), mul_r(R2), mul_r(R3), mul_r(mulmod(R2, R2))};
      __builtin_amdgcn_wave_barrier();  // the previous segment's reads of ml are done
      if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 4; k++) {
#pragma unroll
          for (int i = 0; i < 5; i++) ml[9 * k + i] = Ms[k].v[i];
#pragma unroll
          for (int i = 0; i < 4; i++) ml[9 * k + 5 + i] = Ms[k].s[i];
        }
      }
      __builtin_amdgcn_wave_barrier();
    }
    auto mul_at = [&](int k) {
      MulR M;
#pragma unroll
      for (int i = 0; i < 5; i++) M.v[i] = ml[9 * k + i];
#pragma unroll
      for (int i = 0; i < 4; i++) M.s[i] = ml[9 * k + 5 + i];
      return M;
    };
    // a page = 4 rows of 64 pieces = the 64 ChaCha20 blocks the lanes compute together
    for (uint32_t row0 = 0; row0 < rows; row0 += 4) {
      // the page's ciphertext is loaded first: its latency hides under the page's keystream
      uint4 xin[4];
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const uint32_t boff = (b_lo + (row0 + r) * 64 + lane) * 16;
        xin[r] = make_uint4(0, 0, 0, 0);
        if (row0 + r < rows && boff + 16 <= len) xin[r] = *reinterpret_cast<const uint4*>(src + boff);
      }
      const uint32_t page_byte = (b_lo + row0 * 64) * 16;
      __builtin_amdgcn_wave_barrier();
      if (page_byte < len) {
        uint32_t kb[16];
        chacha_block(key, 1u + (page_byte >> 6) + lane, 0u, n2a, n2b, kb);
        uint4* kd = reinterpret_cast<uint4*>(ks + lane * kKsStride);
        kd[0] = make_uint4(kb[0], kb[1], kb[2], kb[3]);
        kd[1] = make_uint4(kb[4], kb[5], kb[6], kb[7]);
        kd[2] = make_uint4(kb[8], kb[9], kb[10], kb[11]);
        kd[3] = make_uint4(kb[12], kb[13], kb[14], kb[15]);
      }
      __builtin_amdgcn_wave_barrier();
      {
        const uint32_t blk3 = b_lo + (row0 + 3) * 64 + lane;  // the lane's last piece of the page
        if (__all(row0 + 3 < rows && blk3 < nblk_ct && blk3 * 16 + 16 <= len)) {
          // piece r of the page weighs R^(3 - r); the products go into the column sums as each
          // piece is decrypted (no four pieces' limbs held at once)
          uint64_t d[5] = {0, 0, 0, 0, 0};
#pragma unroll
          for (int r = 0; r < 4; r++) {
            const uint32_t boff = (b_lo + (row0 + r) * 64 + lane) * 16;
            const uint32_t q = (uint32_t)r * 64 + lane;
            const uint4 k4 = *reinterpret_cast<const uint4*>(ks + (q >> 2) * kKsStride + (q & 3) * 16);
            const uint4 x = xin[r];
            const uint4 y = make_uint4(x.x ^ k4.x, x.y ^ k4.y, x.z ^ k4.z, x.w ^ k4.w);
            *reinterpret_cast<uint4*>(dst + boff) = y;
            const uint4 c = SEAL ? y : x;
            const L5 m = block_limbs(c.x, c.y, c.z, c.w);
            if (r < 3) {
              mac5(d, m, mul_at(2 - r));
            } else {
#pragma unroll
              for (int i = 0; i < 5; i++) d[i] += m.v[i];
            }
          }
          mac5(d, acc, mul_at(3));
          acc = reduce5(d);
          continue;
        }
      }
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const uint32_t row = row0 + r;
      if (row >= rows) break;
      const uint32_t rb = b_lo + row * 64;  // first block of this row
      const uint32_t blk = rb + lane;
      if (blk < nblk_ct) {
        const uint32_t boff = blk * 16;
        const uint32_t q = (uint32_t)r * 64 + lane;  // piece within the page
        const uint4 k4 = *reinterpret_cast<const uint4*>(ks + (q >> 2) * kKsStride + (q & 3) * 16);
        uint4 x;
        const bool full = boff + 16 <= len;
        if (full) {
          x = xin[r];
        } else {
          uint32_t wv[4] = {0, 0, 0, 0};
          for (uint32_t b = 0; b < len - boff; b++) wv[b >> 2] |= (uint32_t)src[boff + b] << (8 * (b & 3));
          x = make_uint4(wv[0], wv[1], wv[2], wv[3]);
        }
        uint4 y = make_uint4(x.x ^ k4.x, x.y ^ k4.y, x.z ^ k4.z, x.w ^ k4.w);
        if (full) {
          *reinterpret_cast<uint4*>(dst + boff) = y;
        } else {
          const uint32_t rem = len - boff;
          const uint32_t wv[4] = {y.x, y.y, y.z, y.w};
          for (uint32_t b = 0; b < rem; b++) dst[boff + b] = (uint8_t)(wv[b >> 2] >> (8 * (b & 3)));
          // zero the pad bytes of the MAC input
          uint32_t mw[4];
          const uint32_t c[4] = {SEAL ? y.x : x.x, SEAL ? y.y : x.y, SEAL ? y.z : x.z, SEAL ? y.w : x.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const int lo = 4 * i;
            const uint32_t keep = rem >= (uint32_t)(lo + 4) ? 0xffffffffu
                                  : (rem <= (uint32_t)lo ? 0u : ((1u << (8 * (rem - lo))) - 1));
            mw[i] = c[i] & keep;
          }
          if (SEAL) y = make_uint4(mw[0], mw[1], mw[2], mw[3]);
          else x = make_uint4(mw[0], mw[1], mw[2], mw[3]);
        }
        const uint4 m = SEAL ? y : x;
        acc = add5(mulmod(acc, R), block_limbs(m.x, m.y, m.z, m.w));
      } else if (blk == nblk_ct) {
        // length block: le64(aad_len = 0) || le64(ct_len)
        acc = add5(mulmod(acc, R), block_limbs(0u, 0u, len, 0u));
      }
    }
    }
    // rotate so position p = lane holds the lane whose last block has weight r^(64 - p)
    L5 v;
    {
      const int srcl = (int)((lane + nb) & 63);
#pragma unroll
      for (int i = 0; i < 5; i++) v.v[i] = __shfl(acc.v[i], srcl);
    }
#pragma unroll
    for (int k = 0; k < 6; k++) {
      const L5 rk = load_l5(Pp->rpow[k]);
      L5 o;
#pragma unroll
      for (int i = 0; i < 5; i++) o.v[i] = __shfl_down(v.v[i], 1u << k);
      v = carry5(add5(mulmod(v, rk), o));
    }
    L5 tot = mulmod(v, load_l5(Pp->rpow[0]));
#pragma unroll
    for (int i = 0; i < 5; i++) tot.v[i] = bcast(tot.v[i]);

    bool auth_ok = true;
    if (nseg == 1) {
      const uint32_t sv[4] = {Pp->s[0], Pp->s[1], Pp->s[2], Pp->s[3]};
      uint32_t tag[4];
      poly_tag(tot, sv, tag);
      if (SEAL) {
        if (lane < 4) {
          const uint32_t tv = lane == 0 ? tag[0] : lane == 1 ? tag[1] : lane == 2 ? tag[2] : tag[3];
          uint8_t* tp = dst + len + 4 * lane;
          tp[0] = (uint8_t)tv; tp[1] = (uint8_t)(tv >> 8); tp[2] = (uint8_t)(tv >> 16);
          tp[3] = (uint8_t)(tv >> 24);
        }
      } else {
        const bool ok = ((tag[0] ^ Pp->tag[0]) | (tag[1] ^ Pp->tag[1]) | (tag[2] ^ Pp->tag[2]) |
                         (tag[3] ^ Pp->tag[3])) == 0;
        auth_ok = ok;
        if (!ok) {
          // verify-before-release: scrub the speculative plaintext
          for (uint32_t b = lane * 16; b < len; b += 64 * 16) {
            if (b + 16 <= len) *reinterpret_cast<uint4*>(dst + b) = make_uint4(0, 0, 0, 0);
            else for (uint32_t t = b; t < len; t++) dst[t] = 0;
          }
          if (lane == 0) {
            status[f] = CE_ERR_AUTH;
            atomicAdd(&sc.counters[2], 1u);
            atomicMin(&sc.counters[5], f);
          }
        }
      }
    } else if (lane == 0) {
      uint32_t* pp = sc.partials + 5ull * (Pp->extra_base + j);
#pragma unroll
      for (int i = 0; i < 5; i++) pp[i] = tot.v[i];
    }
    if (DEC) {
      // this wave's plaintext stores complete before its lanes read each other's bytes
      __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup");
      __builtin_amdgcn_wave_barrier();
      if (nseg == 1) {
        if (auth_ok) decode_file(da, f, lane);
      } else {
        const uint32_t S = j * kSegBytes;
        seg_record(da, dst, len, S, min(len, S + kSegBytes), lane, rec + 2ull * (Pp->extra_base + j));
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// multi-segment finalize: one wavefront per multi-segment file (grid-stride)
// ----------------------------------------------------------------------------------------
// r^e for any 32-bit e, from r^(2^k) (k <= 6) and further squarings
__device__ L5 rpow_any(const FileParams& P, uint32_t e) {
  L5 acc = {{1, 0, 0, 0, 0}};
  L5 p = load_l5(P.rpow[0]);
  for (int k = 0; k < 32 && (e >> k) != 0; k++) {
    if (k <= 6) p = load_l5(P.rpow[k]);
    else p = mulmod(p, p);
    if (e & (1u << k)) acc = mulmod(acc, p);
  }
  return acc;
}

// The segment partials combine as Horner, acc = acc * r^(blocks of segment j) + p_j, which is
// the sum of p_j * r^(blocks after segment j): lane j takes segment j's term (64 segments a
// round), and a butterfly sums the wave, so a 1 MiB file is not a 65-step dependent chain.
template <bool SEAL>
__global__ __launch_bounds__(256) void k_finalize_multi(uint8_t* __restrict__ out,
                                                        const FileParams* __restrict__ params,
                                                        int32_t* __restrict__ status,
                                                        SegScratch sc) {
  const uint32_t nm = sc.counters[1];
  const uint32_t SB = SEAL ? sc.seg_blocks : kSegBlocks;  // Poly1305 blocks per segment
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * kWavesPerBlock;
  for (uint32_t t = bcast(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); t < nm; t += stride) {
    const uint32_t f = bcast(sc.multi_files[t]);
    const FileParams& P = params[f];
    const uint32_t len = P.len, nseg = P.nseg, base = P.extra_base;
    const uint32_t nblk = ((len + 15) >> 4) + 1;
    // segments j < nseg - 1 are whole: p_j's weight is r^(nblk - (j + 1) S).  Lane l takes
    // j = l, l + 64, ... as a Horner chain in T = r^(64 S) (one mulmod per segment) and scales
    // its sum once by the weight of its last segment; the last segment (weight 1) is added by
    // lane 0.  A 35 MB file (2,200 segments) is then ~35 chain steps per lane, where a power
    // per segment (rpow_any, ~37 mulmods each) made one wave spend ~0.2 ms on it.
    L5 sum = {{0, 0, 0, 0, 0}};
    L5 T = load_l5(P.rpow[6]);  // r^64 -> r^(64 S), only when a lane has a second segment
    if (nseg > 65) {
#pragma unroll 1
      for (uint32_t e = 64; e < 64u * SB; e <<= 1) T = mulmod(T, T);
    }
    if (nseg > 1 + lane) {
      L5 acc = load_l5(sc.partials + 5ull * (base + lane));
      uint32_t jl = lane;
      for (uint32_t j = lane + 64; j + 1 < nseg; j += 64) {
        acc = add5(mulmod(acc, T), load_l5(sc.partials + 5ull * (base + j)));
        jl = j;
      }
      sum = mulmod(carry5(acc), rpow_any(P, nblk - (jl + 1) * SB));
    }
    if (lane == 0) sum = carry5(add5(sum, load_l5(sc.partials + 5ull * (base + nseg - 1))));
#pragma unroll
    for (int k = 0; k < 6; k++) {
      L5 o;
#pragma unroll
      for (int i = 0; i < 5; i++) o.v[i] = __shfl_xor(sum.v[i], 1 << k);
      sum = carry5(add5(sum, o));
    }
    uint32_t tag[4];
    const uint32_t sv[4] = {P.s[0], P.s[1], P.s[2], P.s[3]};
    poly_tag(sum, sv, tag);
    uint8_t* dst = out + P.out_off;
    if (SEAL) {
      if (lane < 16) dst[len + lane] = (uint8_t)(tag[lane >> 2] >> (8 * (lane & 3)));
    } else {
      const bool ok = ((tag[0] ^ P.tag[0]) | (tag[1] ^ P.tag[1]) | (tag[2] ^ P.tag[2]) |
                       (tag[3] ^ P.tag[3])) == 0;
      if (!ok) {
        // verify-before-release: scrub the plaintext (out_off is 16-byte aligned for open)
        for (uint32_t o = lane * 16; o < len; o += 64 * 16) {
          if (o + 16 <= len) *reinterpret_cast<uint4*>(dst + o) = make_uint4(0, 0, 0, 0);
          else for (uint32_t q = o; q < len; q++) dst[q] = 0;
        }
        if (lane == 0) {
          status[f] = CE_ERR_AUTH;
          atomicAdd(&sc.counters[2], 1u);
          atomicMin(&sc.counters[5], f);
        }
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// decode + fold: one wavefront per file
// ----------------------------------------------------------------------------------------
// one wave decodes and folds file f front to back (the general path; k_decode_split's fallback)
__device__ void decode_file(const DecodeArgs& a, uint32_t f, uint32_t lane) {
  {
    const FileParams* Pp = a.params + f;
    const uint8_t* pt = a.pt + Pp->out_off;
    const uint32_t len = Pp->len;
    int32_t st = CE_OK;
    // clear text = VersionBytes(data_version, msgpack(Vec<Op>)) (crdt-enc/src/lib.rs:504-507)
    if (len < 16) st = CE_ERR_PT_LEN;
    else {
      const uint4 dv = *reinterpret_cast<const uint4*>(pt);
      bool found = false;
      for (uint32_t s = 0; s < a.n_supported; s++) {
        const uint4 sv = *reinterpret_cast<const uint4*>(a.supported + 16 * s);
        found |= dv.x == sv.x && dv.y == sv.y && dv.z == sv.z && dv.w == sv.w;
      }
      if (!found) st = CE_ERR_PT_VERSION;
    }
    const bool do_fold = st == CE_OK && (a.apply == nullptr || a.apply[f]);
    // per-lane fold: the last resolved actor is cached (a file's dots are mostly one actor's),
    // the running max for the current slot stays in the lane and is flushed on a slot change;
    // at the end of the file one wave max when every lane holds the same slot
    uint32_t pslot = 0xffffffffu, cslot = 0xffffffffu, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    unsigned long long pbest = 0;
    auto fold_dot = [&](uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3, unsigned long long ctr) {
      uint32_t slot;
      if (cslot != 0xffffffffu && k0 == c0 && k1 == c1 && k2 == c2 && k3 == c3) slot = cslot;
      else {
        slot = lookup_slot1(a.table, a.mask, a.nil_actor, k0, k1, k2, k3);
        if (slot != 0xffffffffu) { c0 = k0; c1 = k1; c2 = k2; c3 = k3; cslot = slot; }
      }
      if (slot == 0xffffffffu) {
        const uint32_t mi = atomicAdd(&a.counters[4], 1u);
        if (mi < a.miss_cap) a.miss_list[mi] = make_uint4(k0, k1, k2, k3);
        a.refold[f] = 1;
      } else if (slot == pslot) {
        pbest = ctr > pbest ? ctr : pbest;
      } else {
        if (pslot != 0xffffffffu) batch_max(&a.batch[pslot], pbest);
        pslot = slot;
        pbest = ctr;
      }
    };
    if (st == CE_OK) {
      const uint8_t* body = pt + 16;
      const uint32_t blen = len - 16;
      Rd r{body, blen, 0};
      uint64_t count = 0;
      if (!rd_array_hdr(r, &count)) st = CE_ERR_DECODE;
      uint32_t pos = (uint32_t)r.i;
      uint64_t remaining = st == CE_OK ? count : 0;
      if (remaining > blen) st = CE_ERR_DECODE, remaining = 0;  // each Dot takes >= 1 byte
      // canonical rmp-serde Dot: 82 a5"actor" c4 10 <16> a7"counter" <uint>  (33 + 1..9 bytes).
      // A round reads 64 candidate Dots at pos + lane L.  L is speculated from the previous round
      // (the first round's from the marker), so the next round's loads are issued before this
      // round's fold; a round whose first Dot does not have length L re-reads the marker.
      uint32_t L = remaining > 0 && pos + 34 <= blen ? dot_len_of_marker(body[pos + 33]) : 0;
      uint4 A = make_uint4(0, 0, 0, 0), B = A, C = A;
      auto load = [&](uint32_t p0, uint64_t rem) {
        const uint32_t cand = p0 + lane * L;
        const bool in = L != 0 && lane < rem && cand + L <= blen;
        const uint8_t* q = body + (in ? cand : 0u);
        A = *reinterpret_cast<const uint4*>(q);
        B = *reinterpret_cast<const uint4*>(q + 16);
        C = *reinterpret_cast<const uint4*>(q + 32);
        return in;
      };
      bool in = load(pos, remaining);
      while (remaining > 0 && st == CE_OK) {
        bool valid = false;
        uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
        unsigned long long ctr = 0;
        if (in) {
          const uint32_t w[12] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, C.x, C.y, C.z, C.w};
          valid = canon_dot(w, L, k0, k1, k2, k3, ctr);
        }
        const unsigned long long vm = __ballot(valid);
        // leading run of valid lanes (ctz of 0 is undefined: all 64 valid -> 64)
        const uint32_t k = vm == ~0ull ? 64u : (uint32_t)__builtin_ctzll(~vm);
        if (k > 0) {
          pos += k * L;
          remaining -= k;
          const bool me = lane < k;
          in = load(pos, remaining);  // next round in flight while this one folds
          if (do_fold && me) fold_dot(k0, k1, k2, k3, ctr);
          continue;
        }
        const uint32_t L2 = pos + 34 <= blen ? dot_len_of_marker(body[pos + 33]) : 0;
        if (L2 != 0 && L2 != L) {  // the Dot length changed: the same position, the new length
          L = L2;
          in = load(pos, remaining);
          continue;
        }
        // general grammar for one element (lane 0), e.g. reordered keys / array form
        int ok = 0;
        uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0;
        unsigned long long gc = 0;
        uint32_t npos = pos;
        if (lane == 0) {
          Rd q{body, blen, pos};
          uint64_t aoff = 0, c = 0;
          ok = parse_dot(q, &aoff, &c);
          if (ok == 1) {
            g0 = ld_le32(body + aoff); g1 = ld_le32(body + aoff + 4);
            g2 = ld_le32(body + aoff + 8); g3 = ld_le32(body + aoff + 12);
            gc = c;
            npos = (uint32_t)q.i;
          }
        }
        ok = __shfl(ok, 0);
        if (ok != 1) { st = CE_ERR_DECODE; break; }
        npos = bcast(npos);
        if (do_fold && lane == 0) fold_dot(g0, g1, g2, g3, gc);
        pos = npos;
        remaining -= 1;
        L = remaining > 0 && pos + 34 <= blen ? dot_len_of_marker(body[pos + 33]) : 0;
        in = load(pos, remaining);
      }
      if (do_fold) {  // flush: one atomicMax per file when the lanes' pending slots agree
        const uint32_t hi = pslot == 0xffffffffu ? 0u : pslot + 1;
        const uint32_t lo = pslot == 0xffffffffu ? 0xffffffffu : pslot + 1;
        uint32_t mx = hi, mn = lo;
        unsigned long long b = pslot == 0xffffffffu ? 0ull : pbest;
#pragma unroll
        for (int d = 32; d >= 1; d >>= 1) {
          const uint32_t omx = (uint32_t)__shfl_xor((int)mx, d), omn = (uint32_t)__shfl_xor((int)mn, d);
          const unsigned long long ob = __shfl_xor(b, d);
          mx = omx > mx ? omx : mx;
          mn = omn < mn ? omn : mn;
          b = ob > b ? ob : b;
        }
        if (mx != 0 && mn == mx) {
          if (lane == 0) batch_max(&a.batch[mx - 1], b);
        } else if (pslot != 0xffffffffu) {
          batch_max(&a.batch[pslot], pbest);
        }
      }
    }
    if (st != CE_OK && lane == 0) {
      a.status[f] = st;
      atomicAdd(&a.counters[3], 1u);
      atomicMin(&a.counters[5], f);
    }
  }
}

__global__ __launch_bounds__(256) void k_decode_dots(DecodeArgs a) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * kWavesPerBlock;
  // large_only: iterate the large-file list of the setup kernel (counters[9])
  const uint32_t nwork = (a.large_only && !a.only) ? *((volatile uint32_t*)&a.counters[9]) : a.n;
  if (a.large_only && !a.only) {
    // the large-file list is pulled one file per wave (counters[15], zeroed before the launch):
    // files run from 4 KiB to MiBs, so a static stride leaves some waves with several big ones
    for (;;) {
      uint32_t w = 0;
      if (lane == 0) w = atomicAdd(&a.counters[15], 1u);
      w = __shfl(w, 0);
      if (w >= nwork) break;
      const uint32_t f = bcast(a.large_list[w]);
      const FileParams* Pp = a.params + f;
      if (Pp->len <= kSmallMax || a.status[f] != CE_OK) continue;
      decode_file(a, f, lane);
    }
    return;
  }
  for (uint32_t w = bcast(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); w < nwork; w += stride) {
    const uint32_t f = w;
    const FileParams* Pp = a.params + f;
    if ((a.only && !a.only[f]) || (a.large_only && Pp->len <= kSmallMax)) continue;
    if (a.status[f] != CE_OK) continue;
    decode_file(a, f, lane);
  }
}

// Multi-page files split over kSplitParts waves (C4's 1 MiB files were one wave each: ~380
// dependent 64-Dot rounds set the kernel's tail).  Part p takes Dots [p*D, (p+1)*D) at byte
// pos0 + p*D*L, assuming every Dot before it is canonical with the first Dot's length L.  That
// only holds once every part has checked its own Dots, so no part folds: each leaves one
// (slot, max) record (its lanes must agree on one actor, no misses), and k_decode_split_apply,
// the next launch on the stream, applies a file's records, or runs decode_file over the whole
// file when any part failed (another Dot length, a non-canonical Dot, a second actor, a miss).
// (A last-finisher counter in one kernel needed two device-scope fences per part: 13x slower.)
__global__ __launch_bounds__(256) void k_decode_split(DecodeArgs a, SplitScratch sp) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * kWavesPerBlock;
  const uint32_t nl = *((volatile uint32_t*)&a.counters[9]);
  for (uint32_t item = bcast(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); item < nl * kSplitParts;
       item += stride) {
    const uint32_t w = item / kSplitParts, part = item % kSplitParts;
    const uint32_t f = bcast(a.large_list[w]);
    const FileParams* Pp = a.params + f;
    if (Pp->len <= kSmallMax || a.status[f] != CE_OK) continue;
    const uint8_t* pt = a.pt + Pp->out_off;
    const uint32_t len = Pp->len;
    // eligibility: supported data version, array header, canonical first Dot length, enough
    // Dots, folded (not gated off); everything else is decode_file's, on part 0
    bool split = len >= 16 && (a.apply == nullptr || a.apply[f]);
    uint32_t count = 0, pos0 = 0, L = 0;
    const uint8_t* body = pt + 16;
    const uint32_t blen = split ? len - 16 : 0;
    if (split) {
      const uint4 dv = *reinterpret_cast<const uint4*>(pt);
      bool found = false;
      for (uint32_t s = 0; s < a.n_supported; s++) {
        const uint4 sv = *reinterpret_cast<const uint4*>(a.supported + 16 * s);
        found |= dv.x == sv.x && dv.y == sv.y && dv.z == sv.z && dv.w == sv.w;
      }
      Rd r{body, blen, 0};
      uint64_t c64 = 0;
      split = found && rd_array_hdr(r, &c64) && c64 <= blen && c64 >= kSplitMinDots;
      if (split) {
        count = (uint32_t)c64;
        pos0 = (uint32_t)r.i;
        L = pos0 + 34 <= blen ? dot_len_of_marker(body[pos0 + 33]) : 0;
        split = L != 0;
      }
    }
    if (!split) {
      if (part == 0) {
        decode_file(a, f, lane);
        if (lane == 0) sp.part[item] = make_uint4(kSplitDone, 0u, 0u, 0u);
      }
      continue;
    }
    const uint32_t D = ((count + kSplitParts - 1) / kSplitParts + 63) & ~63u;
    const uint32_t d0 = min(part * D, count), d1 = min(d0 + D, count);
    bool fail = false;
    uint32_t myslot = 0xffffffffu, cslot = 0xffffffffu, c0 = 0, c1 = 0, c2 = 0, c3 = 0;
    unsigned long long best = 0;
    for (uint32_t i = d0; i < d1; i += 64) {
      const uint32_t k = i + lane;
      const uint64_t cand = pos0 + (uint64_t)k * L;
      const bool in = k < d1 && cand + L <= blen;
      const uint8_t* q = body + (in ? cand : 0u);
      const uint4 A = *reinterpret_cast<const uint4*>(q);
      const uint4 B = *reinterpret_cast<const uint4*>(q + 16);
      const uint4 C = *reinterpret_cast<const uint4*>(q + 32);
      uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
      unsigned long long ctr = 0;
      bool valid = false;
      if (in) {
        const uint32_t wv[12] = {A.x, A.y, A.z, A.w, B.x, B.y, B.z, B.w, C.x, C.y, C.z, C.w};
        valid = canon_dot(wv, L, k0, k1, k2, k3, ctr);
      }
      if (k < d1 && !valid) fail = true;
      if (valid) {
        uint32_t slot;
        if (cslot != 0xffffffffu && k0 == c0 && k1 == c1 && k2 == c2 && k3 == c3) slot = cslot;
        else {
          slot = lookup_slot1(a.table, a.mask, a.nil_actor, k0, k1, k2, k3);
          c0 = k0; c1 = k1; c2 = k2; c3 = k3; cslot = slot;
        }
        if (slot == 0xffffffffu || (myslot != 0xffffffffu && slot != myslot)) fail = true;
        else {
          best = (myslot == 0xffffffffu || ctr > best) ? ctr : best;
          myslot = slot;
        }
      }
    }
    // the wave's record: one slot for all lanes (+1, 0 = no Dots) and the max counter
    uint32_t mx = myslot == 0xffffffffu ? 0u : myslot + 1;
    uint32_t mn = myslot == 0xffffffffu ? 0xffffffffu : myslot + 1;
    unsigned long long bm = best;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint32_t omx = (uint32_t)__shfl_xor((int)mx, d), omn = (uint32_t)__shfl_xor((int)mn, d);
      const unsigned long long ob = __shfl_xor(bm, d);
      mx = omx > mx ? omx : mx;
      mn = omn < mn ? omn : mn;
      bm = ob > bm ? ob : bm;
    }
    const bool wfail = __ballot(fail) != 0 || (mx != 0 && mn != mx);
    if (lane == 0)
      sp.part[item] = make_uint4(wfail ? 0xffffffffu : mx, 0u, (uint32_t)bm, (uint32_t)(bm >> 32));
  }
}

// wave per large file: apply the split parts' records, or decode the file in one wave
__global__ __launch_bounds__(256) void k_decode_split_apply(DecodeArgs a, SplitScratch sp) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t stride = gridDim.x * kWavesPerBlock;
  const uint32_t nl = *((volatile uint32_t*)&a.counters[9]);
  for (uint32_t w = bcast(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); w < nl; w += stride) {
    const uint32_t f = bcast(a.large_list[w]);
    const FileParams* Pp = a.params + f;
    if (Pp->len <= kSmallMax || a.status[f] != CE_OK) continue;
    uint4 rec = make_uint4(0, 0, 0, 0);
    if (lane < kSplitParts) rec = sp.part[(uint64_t)w * kSplitParts + lane];
    if (bcast(rec.x) == kSplitDone) continue;  // decoded in one wave by part 0
    const bool anyfail = __ballot(lane < kSplitParts && rec.x == 0xffffffffu) != 0;
    if (!anyfail) {
      if (lane < kSplitParts && rec.x != 0)
        batch_max(&a.batch[rec.x - 1], (unsigned long long)rec.z | ((unsigned long long)rec.w << 32));
    } else {
      decode_file(a, f, lane);
    }
  }
}

// C4's fused decode, part 2: one wave per multi-segment file after k_finalize_multi (tags
// known).  The file's true Dot grid (header, first Dot length) says which Dots lie wholly inside
// each segment; every segment's record must match it exactly (first offset, count, length, one
// resolved actor), lane j decodes the Dot crossing segment j's end from the plaintext in HBM,
// and the maxima are folded.  Any mismatch -- another Dot length, a non-canonical Dot, a second
// actor, a miss, a grid from a look-alike -- marks the file in redo instead, for k_decode_dots
// (the whole-file decode, launched next over the marked files; decode_file inline here cost
// the common path its registers and a scratch frame).
__global__ __launch_bounds__(256) void k_segdec_apply(DecodeArgs a, SegScratch sc, const uint4* __restrict__ rec) {
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t nm = *((volatile uint32_t*)&sc.counters[1]);
  const uint32_t stride = gridDim.x * kWavesPerBlock;
  // files folded from records, counted per wave and added once per block (one global atomic
  // per file on one word serialised in L2: ~0.18 ms at C4's 16K files)
  __shared__ uint32_t folded[kWavesPerBlock];
  uint32_t n_folded = 0;
  for (uint32_t t = bcast(blockIdx.x * kWavesPerBlock + (threadIdx.x >> 6)); t < nm; t += stride) {
    const uint32_t f = bcast(sc.multi_files[t]);
    const FileParams* Pp = a.params + f;
    if (a.status[f] != CE_OK) continue;
    const uint8_t* pt = a.pt + Pp->out_off;
    const uint32_t len = Pp->len, nseg = Pp->nseg, eb = Pp->extra_base;
    // the first 64 segments' records in one round trip; segment 0's carries the header
    uint4 q0 = make_uint4(0, 0, 0, 0), q1 = q0;
    if (lane < nseg) {
      q0 = rec[2ull * (eb + lane)];
      q1 = rec[2ull * (eb + lane) + 1];
    }
    const uint32_t hok = (uint32_t)__shfl((int)q1.w, 0);
    const bool fold_ok = a.apply == nullptr || a.apply[f];
    if (!hok || !fold_ok) {  // the whole-file decode (k_decode_dots over redo) takes it
      if (lane == 0) {
        a.redo[f] = 1;
        atomicAdd(&a.counters[14], 1u);
      }
      continue;
    }
    const uint32_t hb = (uint32_t)__shfl((int)q0.x, 0), hl = (uint32_t)__shfl((int)q0.w, 0),
                   hc = (uint32_t)__shfl((int)q1.z, 0);
    bool bad = false;
    uint32_t myslot = 0xffffffffu;
    unsigned long long best = 0;
    SlotCache cache;
    auto take = [&](uint32_t sl, unsigned long long v) {
      if (myslot != 0xffffffffu && sl != myslot) bad = true;
      else {
        best = (myslot == 0xffffffffu || v > best) ? v : best;
        myslot = sl;
      }
    };
    for (uint32_t j0 = 0; j0 < nseg; j0 += 64) {
      const uint32_t j = j0 + lane;
      if (j >= nseg) continue;
      const uint32_t S = j * kSegBytes, E = min(len, S + kSegBytes);
      const uint32_t kf = S <= hb ? 0u : (S - hb + hl - 1) / hl;  // first grid Dot starting >= S
      const uint32_t kw = E <= hb ? 0u : (E - hb) / hl;           // grid Dots ending <= E
      const uint32_t ke = min(hc, kw);
      const uint32_t en = ke > kf ? ke - kf : 0u;
      const uint4 r0 = j0 == 0 ? q0 : rec[2ull * (eb + j)], r1 = j0 == 0 ? q1 : rec[2ull * (eb + j) + 1];
      if (r0.y != en || (en != 0 && (r0.x != hb + kf * hl || r0.z == 0xffffffffu || r0.w != hl))) bad = true;
      else if (en != 0 && r0.z != 0) take(r0.z - 1, (unsigned long long)r1.x | ((unsigned long long)r1.y << 32));
      // the grid Dot that starts inside the segment and ends past E
      const uint32_t ps = hb + kw * hl;
      if (E > hb && kw < hc && ps < E && ps >= S) {
        uint32_t w[12], k0, k1, k2, k3;
        unsigned long long ctr;
        dot_window(pt, ps, w);
        if (!canon_dot(w, hl, k0, k1, k2, k3, ctr)) bad = true;
        else {
          const uint32_t sl = cache.get(a, k0, k1, k2, k3);
          if (sl == 0xffffffffu) bad = true;
          else take(sl, ctr);
        }
      }
    }
    if (__ballot(bad) != 0) {
      if (lane == 0) {
        a.redo[f] = 1;
        atomicAdd(&a.counters[14], 1u);
      }
      continue;
    }
    n_folded++;
    uint32_t mx = myslot == 0xffffffffu ? 0u : myslot + 1;
    uint32_t mn = myslot == 0xffffffffu ? 0xffffffffu : myslot + 1;
    unsigned long long bm = myslot == 0xffffffffu ? 0ull : best;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
      const uint32_t omx = (uint32_t)__shfl_xor((int)mx, d), omn = (uint32_t)__shfl_xor((int)mn, d);
      const unsigned long long ob = __shfl_xor(bm, d);
      mx = omx > mx ? omx : mx;
      mn = omn < mn ? omn : mn;
      bm = ob > bm ? ob : bm;
    }
    if (mx != 0 && mn == mx) {
      if (lane == 0) batch_max(&a.batch[mx - 1], bm);
    } else if (myslot != 0xffffffffu) {
      batch_max(&a.batch[myslot], best);
    }
  }
  if (lane == 0) folded[threadIdx.x >> 6] = n_folded;
  __syncthreads();
  if (threadIdx.x == 0) {
    uint32_t tot = 0;
    for (int w = 0; w < kWavesPerBlock; w++) tot += folded[w];
    if (tot) atomicAdd(&a.counters[11], tot);
  }
}

__global__ void k_merge_max(unsigned long long* __restrict__ dst,
                            const unsigned long long* __restrict__ src, uint32_t n) {
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long s = src[i];
    if (s > dst[i]) dst[i] = s;
  }
}

// the same merge, skipped on the device when the batch cannot commit as folded: any auth /
// decode / setup failure ([2] [3] [8]), unregistered actors ([4]), host-parse envelopes ([7]) or
// a batch the device gate could not take ([12]).  The host reads the same counters afterwards and
// takes its slow path exactly when this kernel skipped (no round trip between fold and commit).
__global__ void k_merge_max_if(unsigned long long* __restrict__ dst,
                               const unsigned long long* __restrict__ src, uint32_t n,
                               const uint32_t* __restrict__ counters) {
  if (counters[2] | counters[3] | counters[4] | counters[7] | counters[8] | counters[12]) return;
  for (uint32_t i = blockIdx.x * blockDim.x + threadIdx.x; i < n; i += gridDim.x * blockDim.x) {
    const unsigned long long s = src[i];
    if (s > dst[i]) dst[i] = s;
  }
}


// next_op_versions of a gated batch on the device: nov[wslot[a]] = max(nov, newnov[a]) (lib.rs:
// 537-538), under the same skip condition as k_merge_max_if
__global__ void k_nov_apply(unsigned long long* __restrict__ nov, const uint32_t* __restrict__ wslot,
                            const unsigned long long* __restrict__ newnov, uint32_t m,
                            const uint32_t* __restrict__ counters) {
  if (counters[2] | counters[3] | counters[4] | counters[7] | counters[8] | counters[12]) return;
  for (uint32_t a = blockIdx.x * blockDim.x + threadIdx.x; a < m; a += gridDim.x * blockDim.x)
    atomicMax(&nov[wslot[a]], newnov[a]);
}

// ----------------------------------------------------------------------------------------
// k_serialize_vclock: to_vec_named(StateWrapper) for S = VClock<Uuid> / GCounter<Uuid>
// (crdt-enc/src/lib.rs:336,739-743) straight from the dense device arrays, so a compaction
// needs no state download and no host serializer.  Byte-identical to serialize_state (ce_core.cpp):
//   [prefix16] 82 b0 "next_op_versions" 81 a4 "dots" <map n_nov> {c4 10 <uuid> <uint>}..
//              a5 "state" [81 a5 "inner"] 81 a4 "dots" <map n_st> {..}
// entries in UUID byte order (BTreeMap), zero counters absent.  Workgroup r (1024 lanes) writes
// sorted entries r*1024 + lane (adjacent lanes write adjacent entries), placed by a block scan of
// their lengths; the bytes of the entries before its round it sums itself from all entries (a
// few KB of loads, no inter-workgroup step).  Workgroup 0 writes the headers and the clear length
// to offs[1] (offs[0] = 0) for the seal that follows on the same stream.
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mp_uint_len(unsigned long long v) {
  return v <= 0x7full ? 1u : v <= 0xffull ? 2u : v <= 0xffffull ? 3u : v <= 0xffffffffull ? 5u : 9u;
}
__device__ __forceinline__ uint32_t mp_map_hdr_len(uint32_t n) { return n <= 15 ? 1u : n <= 0xffff ? 3u : 5u; }
__device__ __forceinline__ uint32_t mp_put_map_hdr(uint8_t* o, uint32_t n) {
  if (n <= 15) { o[0] = (uint8_t)(0x80 | n); return 1; }
  if (n <= 0xffff) { o[0] = 0xde; o[1] = (uint8_t)(n >> 8); o[2] = (uint8_t)n; return 3; }
  o[0] = 0xdf; o[1] = (uint8_t)(n >> 24); o[2] = (uint8_t)(n >> 16); o[3] = (uint8_t)(n >> 8); o[4] = (uint8_t)n;
  return 5;
}
__device__ __forceinline__ uint32_t mp_put_str(uint8_t* o, const char* s, uint32_t l) {
  o[0] = (uint8_t)(0xa0 | l);
  for (uint32_t i = 0; i < l; i++) o[1 + i] = (uint8_t)s[i];
  return l + 1;
}
// exclusive block scan over the 1024 lanes (16 waves); *total = the sum
__device__ __forceinline__ uint32_t block_scan_1024(uint32_t v, uint32_t* ws, uint32_t* total) {
  const uint32_t lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  uint32_t x = v;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) {
    const uint32_t y = (uint32_t)__shfl_up((int)x, d);
    if (lane >= (uint32_t)d) x += y;
  }
  if (lane == 63) ws[w] = x;
  __syncthreads();
  uint32_t pre = 0, tot = 0;
#pragma unroll
  for (uint32_t i = 0; i < 16; i++) {
    const uint32_t s = ws[i];
    pre += i < w ? s : 0u;
    tot += s;
  }
  __syncthreads();
  *total = tot;
  return pre + x - v;
}

template <int R>
__global__ __launch_bounds__(1024) void k_serialize_vclock(
    const unsigned long long* __restrict__ nov, const unsigned long long* __restrict__ st,
    const uint32_t* __restrict__ sorted, uint32_t k, const ActorSlot* __restrict__ table,
    int gcounter, const uint8_t* __restrict__ prefix16, uint8_t* __restrict__ out,
    unsigned long long* __restrict__ offs) {
  __shared__ uint32_t ws[16];
  const uint32_t t = threadIdx.x;
  // R rounds per chunk held in registers: every load of a chunk is issued before any is used
  // (one latency per chunk, not three dependent ones per round).  k <= 1024 R: one chunk, the
  // registers also serve the write pass.
  const uint32_t rounds = (k + 1023) / 1024;
  uint32_t sl[R];
  unsigned long long nv[R], sv[R];
  auto load_chunk = [&](uint32_t r0) {
#pragma unroll
    for (int r = 0; r < R; r++) {
      const uint32_t i = (r0 + r) * 1024 + t;
      sl[r] = i < k ? sorted[i] : 0xffffffffu;
    }
#pragma unroll
    for (int r = 0; r < R; r++) {
      nv[r] = sl[r] != 0xffffffffu ? nov[sl[r]] : 0ull;
      sv[r] = sl[r] != 0xffffffffu ? st[sl[r]] : 0ull;
    }
  };
  // pass 1 (every workgroup, over all entries): entry counts and bytes of both maps, and the
  // bytes of the entries before this workgroup's round (counts packed in 16-bit halves when
  // they fit: <= 1024 R each)
  const uint32_t me = blockIdx.x;  // the round this workgroup writes
  uint32_t cnt = 0, bn = 0, bs = 0, pn = 0, ps = 0;
  for (uint32_t r0 = 0; r0 < rounds; r0 += R) {
    load_chunk(r0);
#pragma unroll
    for (int r = 0; r < R; r++) {
      cnt += (nv[r] != 0 ? 1u : 0u) + (sv[r] != 0 ? 0x10000u : 0u);
      const uint32_t ln = nv[r] != 0 ? 18u + mp_uint_len(nv[r]) : 0u;
      const uint32_t ls = sv[r] != 0 ? 18u + mp_uint_len(sv[r]) : 0u;
      bn += ln;
      bs += ls;
      if (r0 + r < me) { pn += ln; ps += ls; }
    }
  }
  uint32_t tc, tbn, tbs, tpn, tps;
  (void)block_scan_1024(cnt, ws, &tc);
  (void)block_scan_1024(bn, ws, &tbn);
  (void)block_scan_1024(bs, ws, &tbs);
  (void)block_scan_1024(pn, ws, &tpn);
  (void)block_scan_1024(ps, ws, &tps);
  uint32_t cn = tc & 0xffff, cs = tc >> 16;
  if (rounds > R) {  // counts can pass 16 bits: recount exactly
    uint32_t a = 0, b = 0;
    for (uint32_t r0 = 0; r0 < rounds; r0 += R) {
      load_chunk(r0);
#pragma unroll
      for (int r = 0; r < R; r++) { a += nv[r] != 0; b += sv[r] != 0; }
    }
    (void)block_scan_1024(a, ws, &cn);
    (void)block_scan_1024(b, ws, &cs);
  }
  const uint32_t pl = prefix16 ? 16u : 0u;
  const uint32_t nov_at = pl + 24 + mp_map_hdr_len(cn);                 // first nov entry
  const uint32_t st_hdr = nov_at + tbn;                                  // "state" ...
  const uint32_t st_at = st_hdr + 6 + (gcounter ? 7u : 0u) + 6 + mp_map_hdr_len(cs);
  if (me == 0 && t == 0) {
    uint8_t* o = out;
    for (uint32_t i = 0; i < pl; i++) *o++ = prefix16[i];
    *o++ = 0x82;
    o += mp_put_str(o, "next_op_versions", 16);
    *o++ = 0x81;
    o += mp_put_str(o, "dots", 4);
    o += mp_put_map_hdr(o, cn);
    o = out + st_hdr;
    o += mp_put_str(o, "state", 5);
    if (gcounter) {
      *o++ = 0x81;
      o += mp_put_str(o, "inner", 5);
    }
    *o++ = 0x81;
    o += mp_put_str(o, "dots", 4);
    o += mp_put_map_hdr(o, cs);
    offs[0] = 0;
    offs[1] = st_at + tbs;
  }
  // one entry c4 10 <uuid16> <uint>: 19..27 bytes assembled as 7 little-endian dwords, stored
  // as unaligned dwords + the 1..3 trailing bytes (a third of the byte stores; adjacent entries
  // never share a dword store)
  auto put = [&](uint32_t at, const ActorSlot& a, unsigned long long v) {
    const uint32_t ul = mp_uint_len(v);
    const uint32_t nb = ul - 1;  // big-endian payload bytes after the marker
    const unsigned long long be = nb ? __builtin_bswap64(v) >> (8 * (8 - nb)) : 0ull;
    const uint32_t mk = ul == 2 ? 0xccu : ul == 3 ? 0xcdu : ul == 5 ? 0xceu : 0xcfu;
    const unsigned long long lo = ul == 1 ? v : (mk | (be << 8));
    const uint32_t hi = ul == 9 ? (uint32_t)(be >> 56) : 0u;
    const uint32_t t0 = (uint32_t)lo, t1 = (uint32_t)(lo >> 32);
    uint32_t w[7];
    w[0] = 0x10c4u | (a.k[0] << 16);
    w[1] = (a.k[0] >> 16) | (a.k[1] << 16);
    w[2] = (a.k[1] >> 16) | (a.k[2] << 16);
    w[3] = (a.k[2] >> 16) | (a.k[3] << 16);
    w[4] = (a.k[3] >> 16) | (t0 << 16);
    w[5] = (t0 >> 16) | (t1 << 16);
    w[6] = (t1 >> 16) | (hi << 16);
    const uint32_t len = 18 + ul, nd = len >> 2;
    uint8_t* o = out + at;
#pragma unroll
    for (uint32_t q = 0; q < 7; q++)
      if (q < nd) *reinterpret_cast<uint32_t*>(o + 4 * q) = w[q];
    const uint32_t tail = w[nd < 7 ? nd : 6];
    for (uint32_t b = 4 * nd; b < len; b++) o[b] = (uint8_t)(tail >> (8 * (b & 3)));
  };
  // pass 2: this workgroup's round; both maps' entry lengths scanned at once (16-bit halves:
  // <= 27 x 1024)
  {
    const uint32_t i = me * 1024 + t;
    const uint32_t slot = i < k ? sorted[i] : 0xffffffffu;
    const unsigned long long vn = slot != 0xffffffffu ? nov[slot] : 0ull;
    const unsigned long long vs = slot != 0xffffffffu ? st[slot] : 0ull;
    const uint32_t ln = vn != 0 ? 18u + mp_uint_len(vn) : 0u;
    const uint32_t ls = vs != 0 ? 18u + mp_uint_len(vs) : 0u;
    ActorSlot a;
    if (ln | ls) a = table[slot];
    uint32_t tot;
    const uint32_t at = block_scan_1024(ln | (ls << 16), ws, &tot);
    if (ln) put(nov_at + tpn + (at & 0xffff), a, vn);
    if (ls) put(st_at + tps + (at >> 16), a, vs);
  }
}

// ----------------------------------------------------------------------------------------
// launchers
// ----------------------------------------------------------------------------------------
hipError_t launch_open_setup(hipStream_t s, const uint8_t* blob, const uint64_t* offs, uint32_t n,
                             bool outer, DevKey key, int32_t key_status, FileParams* params,
                             int32_t* status, SegScratch sc, PolyAux* aux) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_open_setup, dim3((n + 255) / 256), dim3(256), 0, s, blob, offs, n,
                     outer ? 1 : 0, key, key_status, params, status, sc, aux);
  return hipGetLastError();
}

__global__ void k_fill(FillArgs a) {
  const uint32_t r = blockIdx.y;
  if ((int)r == a.n) {  // the counter block
    if (blockIdx.x == 0 && threadIdx.x < 16)
      a.counters[threadIdx.x] = (threadIdx.x == 5 || threadIdx.x == 13) ? 0xffffffffu : 0u;
    return;
  }
  const FillRange f = a.r[r];
  const uint64_t t0 = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x, ts = (uint64_t)gridDim.x * blockDim.x;
  // 16-byte stores over the aligned body (a table reset is tens of MB: one dword per lane and
  // trip was ~2.4 TB/s), dwords at the ends
  const uint64_t head = ((16 - (reinterpret_cast<uintptr_t>(f.p) & 15)) & 15) / 4;
  const bool vec = (reinterpret_cast<uintptr_t>(f.p) & 3) == 0 &&
                   (!f.src || ((reinterpret_cast<uintptr_t>(f.src) ^ reinterpret_cast<uintptr_t>(f.p)) & 15) == 0) &&
                   f.words > head + 4;
  if (!vec) {
    for (uint64_t i = t0; i < f.words; i += ts) f.p[i] = f.src ? f.src[i] : f.value;
    return;
  }
  const uint64_t body = (f.words - head) / 4, tail0 = head + 4 * body;
  uint4* p4 = reinterpret_cast<uint4*>(f.p + head);
  if (f.src) {
    const uint4* s4 = reinterpret_cast<const uint4*>(f.src + head);
    for (uint64_t i = t0; i < body; i += ts) p4[i] = s4[i];
  } else {
    const uint4 v = make_uint4(f.value, f.value, f.value, f.value);
    for (uint64_t i = t0; i < body; i += ts) p4[i] = v;
  }
  if (t0 < head) f.p[t0] = f.src ? f.src[t0] : f.value;
  if (t0 < f.words - tail0) f.p[tail0 + t0] = f.src ? f.src[tail0 + t0] : f.value;
}

// A compaction's sealed-file length -> a mapped pinned word, behind the seal on its stream: the
// serializer's clear length at clear_len_at -> the file's total (~0: it would not fit in cap;
// ~1: the serializer overran its bound).  One lane; the host reads the word after the seal's
// event and sizes the download by it.
__global__ void k_publish_sealed_len(const uint64_t* clear_len_at, uint64_t bound, uint64_t cap, uint64_t* len_out) {
  const uint64_t cl = *clear_len_at;
  const uint64_t total = 16 + sealed_len(cl);
  *reinterpret_cast<volatile uint64_t*>(len_out) = cl > bound ? ~1ull : total > cap ? ~0ull : total;
}

// n counter words -> mapped pinned memory, then the generation word after them (the host polls
// it): one wave; the fence orders every lane's stores before lane 0's generation store
__global__ void k_publish_words(const uint32_t* src, uint32_t n, uint32_t* dst, uint32_t gen) {
  if (threadIdx.x < n) reinterpret_cast<volatile uint32_t*>(dst)[threadIdx.x] = src[threadIdx.x];
  __threadfence_system();
  if (threadIdx.x == 0) reinterpret_cast<volatile uint32_t*>(dst)[n] = gen;
}

hipError_t launch_publish_words(hipStream_t s, const uint32_t* src, uint32_t n, uint32_t* dst, uint32_t gen) {
  if (n > 64) return hipErrorInvalidValue;
  hipLaunchKernelGGL(k_publish_words, dim3(1), dim3(64), 0, s, src, n, dst, gen);
  return hipGetLastError();
}

hipError_t launch_publish_sealed_len(hipStream_t s, const uint64_t* clear_len_at, uint64_t bound, uint64_t cap,
                                     uint64_t* len_out) {
  hipLaunchKernelGGL(k_publish_sealed_len, dim3(1), dim3(1), 0, s, clear_len_at, bound, cap, len_out);
  return hipGetLastError();
}

hipError_t launch_fill(hipStream_t s, const FillArgs& a) {
  uint64_t mx = 16;
  for (int i = 0; i < a.n; i++) mx = a.r[i].words > mx ? a.r[i].words : mx;
  const uint32_t gx = (uint32_t)std::min<uint64_t>((mx / 4 + 255) / 256, 1024);
  hipLaunchKernelGGL(k_fill, dim3(gx, a.n + (a.counters ? 1 : 0)), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_seal_setup(hipStream_t s, const uint8_t* clear, const uint64_t* offs, uint32_t n,
                             const uint8_t* outer_version, const uint8_t* nonces, uint8_t* out,
                             const uint64_t* out_offs, DevKey key, FileParams* params,
                             SegScratch sc) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_seal_setup, dim3((n + 255) / 256), dim3(256), 0, s, clear, offs, n,
                     outer_version, nonces, out, out_offs, key, params, sc);
  return hipGetLastError();
}

hipError_t launch_segments(hipStream_t s, bool seal, const uint8_t* in, uint8_t* out,
                           const FileParams* params, uint32_t n, int32_t* status, SegScratch sc,
                           uint32_t grid_waves, bool skip_small) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = (grid_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  if (seal)
    hipLaunchKernelGGL((k_segments<true, false>), dim3(blocks), dim3(256), 0, s, in, out, params, n,
                       status, sc, 0, DecodeArgs{}, (uint4*)nullptr);
  else
    hipLaunchKernelGGL((k_segments<false, false>), dim3(blocks), dim3(256), 0, s, in, out, params, n,
                       status, sc, skip_small ? 1 : 0, DecodeArgs{}, (uint4*)nullptr);
  return hipGetLastError();
}

hipError_t launch_segments_decode(hipStream_t s, const uint8_t* in, uint8_t* out, const DecodeArgs& da,
                                  SegScratch sc, uint32_t grid_waves, uint4* rec) {
  if (da.n == 0) return hipSuccess;
  const uint32_t blocks = (grid_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL((k_segments<false, true>), dim3(blocks), dim3(256), 0, s, in, out, da.params, da.n,
                     da.status, sc, 1, da, rec);
  return hipGetLastError();
}

hipError_t launch_segdec_apply(hipStream_t s, const DecodeArgs& a, SegScratch sc, const uint4* rec, uint32_t n_large) {
  if (n_large == 0) return hipSuccess;
  const uint32_t w = min(n_large, 256u * 32u);
  hipLaunchKernelGGL(k_segdec_apply, dim3((w + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, s, a, sc, rec);
  return hipGetLastError();
}

hipError_t launch_finalize_multi(hipStream_t s, bool seal, uint8_t* out, const FileParams* params,
                                 int32_t* status, SegScratch sc, uint32_t n) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = min((n + kWavesPerBlock - 1) / kWavesPerBlock, 1024u);
  if (seal)
    hipLaunchKernelGGL(k_finalize_multi<true>, dim3(blocks), dim3(256), 0, s, out, params, status, sc);
  else
    hipLaunchKernelGGL(k_finalize_multi<false>, dim3(blocks), dim3(256), 0, s, out, params, status, sc);
  return hipGetLastError();
}

hipError_t launch_decode_dots(hipStream_t s, const DecodeArgs& a, uint32_t grid_waves) {
  if (a.n == 0) return hipSuccess;
  const uint32_t blocks = (grid_waves + kWavesPerBlock - 1) / kWavesPerBlock;
  hipLaunchKernelGGL(k_decode_dots, dim3(blocks), dim3(256), 0, s, a);
  return hipGetLastError();
}

hipError_t launch_decode_split(hipStream_t s, const DecodeArgs& a, SplitScratch sp, uint32_t n_large) {
  if (n_large == 0) return hipSuccess;
  const uint32_t waves = min(n_large * kSplitParts, 256u * 32u);
  hipLaunchKernelGGL(k_decode_split, dim3((waves + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, s, a, sp);
  const uint32_t w2 = min(n_large, 256u * 32u);
  hipLaunchKernelGGL(k_decode_split_apply, dim3((w2 + kWavesPerBlock - 1) / kWavesPerBlock), dim3(256), 0, s, a, sp);
  return hipGetLastError();
}

hipError_t launch_merge_max(hipStream_t s, unsigned long long* dst, const unsigned long long* src,
                            uint32_t n) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = min((n + 255) / 256, 1024u);
  hipLaunchKernelGGL(k_merge_max, dim3(blocks), dim3(256), 0, s, dst, src, n);
  return hipGetLastError();
}

hipError_t launch_merge_max_if(hipStream_t s, unsigned long long* dst, const unsigned long long* src,
                               uint32_t n, const uint32_t* counters) {
  if (n == 0) return hipSuccess;
  const uint32_t blocks = min((n + 255) / 256, 1024u);
  hipLaunchKernelGGL(k_merge_max_if, dim3(blocks), dim3(256), 0, s, dst, src, n, counters);
  return hipGetLastError();
}

// diagnostics (ce_ctx_clock_probe): one wave per block reads the shader cycle counter against
// the 100 MHz reference clock every `ticks` reference ticks and stores each interval's
// (cycles, ticks) through lanes 0 and 1.  Launched beside other work, it measures the clock that
// work runs at (the blocks land on the XCDs round-robin).
__global__ __launch_bounds__(64) void k_clock_probe(unsigned long long* out, uint32_t samples,
                                                    uint32_t ticks) {
  const uint32_t lane = threadIdx.x;
  unsigned long long c0 = __builtin_amdgcn_s_memtime();
  unsigned long long r0 = __builtin_amdgcn_s_memrealtime();
  for (uint32_t k = 0; k < samples; k++) {
    unsigned long long r = r0;
    while (r - r0 < ticks) {
      __builtin_amdgcn_s_sleep(2);
      r = __builtin_amdgcn_s_memrealtime();
    }
    const unsigned long long c = __builtin_amdgcn_s_memtime();
    if (lane < 2) out[2ull * ((unsigned long long)blockIdx.x * samples + k) + lane] = lane ? r - r0 : c - c0;
    c0 = c;
    r0 = r;
  }
}

hipError_t launch_clock_probe(hipStream_t s, unsigned long long* out, uint32_t blocks,
                              uint32_t samples, uint32_t ticks) {
  hipLaunchKernelGGL(k_clock_probe, dim3(blocks), dim3(64), 0, s, out, samples, ticks);
  return hipGetLastError();
}

hipError_t launch_nov_apply(hipStream_t s, unsigned long long* nov, const uint32_t* wslot,
                            const unsigned long long* newnov, uint32_t m, const uint32_t* counters) {
  if (m == 0) return hipSuccess;
  hipLaunchKernelGGL(k_nov_apply, dim3(min((m + 255) / 256, 256u)), dim3(256), 0, s, nov,
                     wslot, newnov, m, counters);
  return hipGetLastError();
}

__global__ void k_compact_prologue(uint8_t* args, CompactArgs ca, uint32_t* seal_counters,
                                   unsigned long long* nov, const uint32_t* wslot,
                                   const unsigned long long* newnov, uint32_t m, const uint32_t* counters,
                                   unsigned long long* __restrict__ merge_dst,
                                   const unsigned long long* __restrict__ merge_src, uint32_t merge_n) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t < 24) {  // offs[0] = 0, offs[1] = 0 (the serializer writes the clear length), out_offs[0] = 0
    args[t] = 0;
  } else if (t < 48) {
    args[t] = ca.nonce[t - 24];
  } else if (t < 64) {
    args[t] = ca.outer[t - 48];
  } else if (t < 80) {
    args[t] = ca.prefix[t - 64];
  } else if (t < 96) {
    const uint32_t w = t - 80;
    seal_counters[w] = (w == 5 || w == 13) ? 0xffffffffu : 0u;
  }
  if ((m == 0 && merge_n == 0) ||
      (counters[2] | counters[3] | counters[4] | counters[7] | counters[8] | counters[12]))
    return;
  const uint32_t stride = gridDim.x * blockDim.x;
  for (uint32_t a = t; a < m; a += stride) atomicMax(&nov[wslot[a]], newnov[a]);
  for (uint32_t i = t; i < merge_n; i += stride) {  // the ingest's commit (k_merge_max_if)
    const unsigned long long v = merge_src[i];
    if (v > merge_dst[i]) merge_dst[i] = v;
  }
}

hipError_t launch_compact_prologue(hipStream_t s, uint8_t* args, const CompactArgs& ca, uint32_t* seal_counters,
                                   unsigned long long* nov, const uint32_t* wslot,
                                   const unsigned long long* newnov, uint32_t m, const uint32_t* counters,
                                   unsigned long long* merge_dst, const unsigned long long* merge_src,
                                   uint32_t merge_n) {
  const uint32_t work = m > merge_n ? m : merge_n;
  const uint32_t blocks = work > 96 ? min((work + 255) / 256, 256u) : 1u;
  hipLaunchKernelGGL(k_compact_prologue, dim3(blocks), dim3(256), 0, s, args, ca, seal_counters, nov, wslot,
                     newnov, m, counters, merge_dst, merge_src, merge_n);
  return hipGetLastError();
}

__global__ void k_tail_pack(uint8_t* dst, const unsigned long long* src_len, const uint32_t* counters,
                            const unsigned long long* newnov, uint32_t m) {
  const uint32_t t = blockIdx.x * blockDim.x + threadIdx.x;
  if (t == 0) *reinterpret_cast<unsigned long long*>(dst) = *src_len;
  if (t < 16) reinterpret_cast<uint32_t*>(dst + 8)[t] = counters[t];
  auto* nn = reinterpret_cast<unsigned long long*>(dst + 72);
  for (uint32_t a = t; a < m; a += gridDim.x * blockDim.x) nn[a] = newnov[a];
}

hipError_t launch_tail_pack(hipStream_t s, uint8_t* dst, const unsigned long long* src_len,
                            const uint32_t* counters, const unsigned long long* newnov, uint32_t m) {
  const uint32_t blocks = m > 256 ? min((m + 255) / 256, 64u) : 1u;
  hipLaunchKernelGGL(k_tail_pack, dim3(blocks), dim3(256), 0, s, dst, src_len, counters, newnov, m);
  return hipGetLastError();
}

static constexpr uint32_t kGatherBatch = 16;
struct GatherBatch {
  GatherRange r[kGatherBatch];
};
// blockIdx.y = range; the blocks of a range stride over its bytes, 16 at a time where source and
// destination share an alignment, byte by byte at the edges otherwise
__global__ void k_gather_ranges(uint8_t* __restrict__ dst, GatherBatch b) {
  const GatherRange g = b.r[blockIdx.y];
  uint8_t* d = dst + g.dst_off;
  const uint64_t tid = blockIdx.x * (uint64_t)blockDim.x + threadIdx.x;
  const uint64_t nt = (uint64_t)gridDim.x * blockDim.x;
  const uint64_t mis = (16 - ((uintptr_t)g.src & 15)) & 15;
  if ((((uintptr_t)g.src ^ (uintptr_t)d) & 15) == 0 && g.len > mis + 16) {
    const uint64_t head = mis, body = (g.len - head) & ~15ull;
    for (uint64_t i = tid; i < head; i += nt) d[i] = g.src[i];
    const uint4* s4 = reinterpret_cast<const uint4*>(g.src + head);
    uint4* d4 = reinterpret_cast<uint4*>(d + head);
    for (uint64_t i = tid; i < body / 16; i += nt) d4[i] = s4[i];
    for (uint64_t i = head + body + tid; i < g.len; i += nt) d[i] = g.src[i];
  } else {
    for (uint64_t i = tid; i < g.len; i += nt) d[i] = g.src[i];
  }
}

hipError_t launch_gather_ranges(hipStream_t s, uint8_t* dst, const GatherRange* r, uint32_t n) {
  for (uint32_t i0 = 0; i0 < n; i0 += kGatherBatch) {
    GatherBatch b{};
    const uint32_t k = min(n - i0, kGatherBatch);
    uint64_t mx = 0;
    for (uint32_t i = 0; i < k; i++) {
      b.r[i] = r[i0 + i];
      mx = b.r[i].len > mx ? b.r[i].len : mx;
    }
    if (mx == 0) continue;
    const uint32_t blocks = (uint32_t)std::min<uint64_t>((mx + 16ull * 256 - 1) / (16ull * 256), 256ull);
    hipLaunchKernelGGL(k_gather_ranges, dim3(blocks, k), dim3(256), 0, s, dst, b);
  }
  return hipGetLastError();
}

__global__ void k_state_heads(const FileParams* __restrict__ params, const int32_t* __restrict__ status,
                              const uint8_t* __restrict__ out, uint32_t n, uint8_t* __restrict__ dst) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  const int32_t st = status[i];
  const FileParams& P = params[i];
  uint32_t w[8] = {(uint32_t)st, P.len, (uint32_t)P.out_off, (uint32_t)(P.out_off >> 32), 0, 0, 0, 0};
  if (st == CE_OK && P.len >= 16) {
    const uint8_t* v = out + P.out_off;  // 16-byte aligned (open)
    const uint4 q = *reinterpret_cast<const uint4*>(v);
    w[4] = q.x; w[5] = q.y; w[6] = q.z; w[7] = q.w;
  }
  uint4* o = reinterpret_cast<uint4*>(dst + 32ull * i);
  o[0] = make_uint4(w[0], w[1], w[2], w[3]);
  o[1] = make_uint4(w[4], w[5], w[6], w[7]);
}

hipError_t launch_state_heads(hipStream_t s, const FileParams* params, const int32_t* status,
                              const uint8_t* out, uint32_t n, uint8_t* dst) {
  if (n == 0) return hipSuccess;
  hipLaunchKernelGGL(k_state_heads, dim3((n + 255) / 256), dim3(256), 0, s, params, status, out, n, dst);
  return hipGetLastError();
}

hipError_t launch_serialize_vclock(hipStream_t s, const unsigned long long* nov,
                                  const unsigned long long* st, const uint32_t* sorted, uint32_t k,
                                  const ActorSlot* table, bool gcounter, const uint8_t* prefix16,
                                  uint8_t* out, unsigned long long* offs) {
  // one workgroup per 1024 sorted entries (at least one: the headers)
  const uint32_t rounds = k ? (k + 1023) / 1024 : 1;
  hipLaunchKernelGGL(k_serialize_vclock<4>, dim3(rounds), dim3(1024), 0, s, nov, st, sorted, k, table,
                     gcounter ? 1 : 0, prefix16, out, offs);
  return hipGetLastError();
}

}  // namespace ce
