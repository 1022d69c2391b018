// ce_fused.hip -- the C2 hot loop: open + decode + fold of single-page op files in one kernel,
// and the device version gate.
//
// k_open_fold_small<LPF>: a wavefront handles 64/LPF files at once, LPF lanes per file.
//   1. the file's ciphertext pieces (16 B, coalesced per file) are loaded into registers first,
//      so their latency hides under step 2;
//   2. each lane computes 64/LPF ChaCha20 blocks of the page (counter 1 + block) into LDS;
//   3. piece by piece: keystream from LDS (transposed), plaintext written back over the
//      consumed keystream (LDS), Poly1305 as an LPF-way strided Horner in r^LPF;
//   4. log2(LPF)-level cross-lane tree in r^(2^k) inside the lane group, tag compare
//      (xchacha lib.rs:92-97) -- a failing file folds nothing;
//   5. the plaintext never leaves LDS: VersionBytes data-version check (crdt-enc/src/lib.rs:
//      504-505) and rmp-serde Vec<Dot<Uuid>> decode (lib.rs:507), LPF candidate Dots per round
//      speculating on the canonical encoding (general grammar by the group leader otherwise);
//   6. dots of files the gate applies are max-folded into the batch state (VClock::apply),
//      one pending (slot, max) per lane group -> one atomicMax per file for an actor's own ops.
// Poly1305 tree cost per file falls from 7 mulmods (64 lanes/file) to 5/4 (16 lanes/file).
#include <algorithm>

#include "ce_device.h"

namespace ce {

static constexpr uint32_t kRegion = 64 * kKsStride;  // 5120 B of LDS per file in flight

template <int LPF>
struct FusedCfg {
  static constexpr int F = 64 / LPF;                       // files per wave
  static constexpr int WPB = LPF == 16 ? 2 : 4;            // waves per block
  static constexpr int LOG = LPF == 16 ? 4 : LPF == 32 ? 5 : 6;
  static constexpr int ROWS = (256 + 1 + LPF - 1) / LPF;   // Horner steps for a full page
  static constexpr int WAVES_PER_SIMD = LPF == 16 ? 2 : LPF == 32 ? 4 : 8;  // LDS-limited
};

struct GroupFold {
  uint32_t slot;
  unsigned long long best;
};

template <int LPF>
__device__ __forceinline__ void fold_group(const DecodeArgs& a, uint32_t f, bool active,
                                           uint32_t k0, uint32_t k1, uint32_t k2, uint32_t k3,
                                           unsigned long long ctr, GroupFold& gf, uint32_t grp,
                                           uint32_t sub) {
  constexpr unsigned long long GM = LPF == 64 ? ~0ull : ((1ull << LPF) - 1);
  uint32_t slot = 0xffffffffu;
  if (active) {
    slot = lookup_slot(a.table, a.mask, k0, k1, k2, k3);
    if (slot == 0xffffffffu) {
      const uint32_t mi = atomicAdd(&a.counters[4], 1u);
      if (mi < a.miss_cap) a.miss_list[mi] = make_uint4(k0, k1, k2, k3);
      a.refold[f] = 1;
    }
  }
  const bool live = active && slot != 0xffffffffu;
  const unsigned long long gb = (__ballot(live) >> (grp * LPF)) & GM;
  const uint32_t first = grp * LPF + (uint32_t)__builtin_ctzll(gb | (1ull << (LPF - 1)));
  const uint32_t s0 = __shfl(slot, first);
  const bool same = ((__ballot(live && slot != s0) >> (grp * LPF)) & GM) == 0;
  if (same && gb != 0) {
    unsigned long long v = live ? ctr : 0ull;
#pragma unroll
    for (int d = LPF / 2; d >= 1; d >>= 1) {
      const unsigned long long o = __shfl_xor(v, d);
      v = o > v ? o : v;
    }
    if (gf.slot != s0) {
      if (gf.slot != 0xffffffffu && sub == 0) atomicMax(&a.batch[gf.slot], gf.best);
      gf.slot = s0;
      gf.best = v;
    } else if (v > gf.best) {
      gf.best = v;
    }
  } else if (live) {
    atomicMax(&a.batch[slot], ctr);
  }
}

template <int LPF>
__global__ __launch_bounds__(FusedCfg<LPF>::WPB * 64, FusedCfg<LPF>::WAVES_PER_SIMD)
void k_open_fold_small(DecodeArgs a) {
  using C = FusedCfg<LPF>;
  constexpr int F = C::F;
  constexpr int PPL = 256 / LPF;  // ciphertext pieces per lane (one page)
  __shared__ __attribute__((aligned(16))) uint8_t lds[C::WPB * F * kRegion];
  const uint32_t lane = threadIdx.x & 63;
  const uint32_t wib = threadIdx.x >> 6;
  const uint32_t grp = lane / LPF, sub = lane % LPF;
  uint8_t* fl = lds + (wib * F + grp) * kRegion;
  const uint32_t ngroups = (a.n + F - 1) / F;
  const uint32_t stride = gridDim.x * C::WPB;

  for (uint32_t g = bcast(blockIdx.x * C::WPB + wib); g < ngroups; g += stride) {
    const uint32_t f = g * F + grp;
    bool act = f < a.n;
    if (act && a.only) act = a.only[f] != 0;
    const FileParams* Pp = a.params + (act ? f : 0);
    if (act) act = a.status[f] == CE_OK && Pp->len <= kSmallMax;
    const uint32_t len = act ? Pp->len : 0u;
    const uint32_t nblk_ct = (len + 15) >> 4;
    const uint32_t nb = nblk_ct + 1;
    const uint8_t* src = a.blob + (act ? Pp->in_off : 0);

    // 1) ciphertext pieces -> registers (issued first: latency hides under the ChaCha20)
    uint4 ct[PPL];
#pragma unroll
    for (int j = 0; j < PPL; j++) {
      const uint32_t blk = sub + LPF * j;
      const uint32_t boff = blk * 16;
      if (act && boff + 16 <= len) ct[j] = *reinterpret_cast<const uint4*>(src + boff);
      else if (act && boff < len) {
        uint32_t wv[4] = {0, 0, 0, 0};
        for (uint32_t b = 0; b < len - boff; b++) wv[b >> 2] |= (uint32_t)src[boff + b] << (8 * (b & 3));
        ct[j] = make_uint4(wv[0], wv[1], wv[2], wv[3]);
      } else ct[j] = make_uint4(0, 0, 0, 0);
    }

    // 2) keystream: lane computes blocks sub + LPF*k (ChaCha20 counter 1 + block)
    uint32_t key[8];
#pragma unroll
    for (int i = 0; i < 8; i++) key[i] = act ? Pp->subkey[i] : 0u;
    const uint32_t n2a = act ? Pp->n2[0] : 0u, n2b = act ? Pp->n2[1] : 0u;
    __builtin_amdgcn_wave_barrier();
#pragma unroll
    for (int k = 0; k < F; k++) {
      const uint32_t b = sub + LPF * k;
      if (act && b * 64 < len) {
        uint32_t kb[16];
        chacha_block(key, 1u + b, 0u, n2a, n2b, kb);
        uint4* kd = reinterpret_cast<uint4*>(fl + b * kKsStride);
        kd[0] = make_uint4(kb[0], kb[1], kb[2], kb[3]);
        kd[1] = make_uint4(kb[4], kb[5], kb[6], kb[7]);
        kd[2] = make_uint4(kb[8], kb[9], kb[10], kb[11]);
        kd[3] = make_uint4(kb[12], kb[13], kb[14], kb[15]);
      }
    }
    __builtin_amdgcn_wave_barrier();

    // 3) XOR, plaintext into LDS (over consumed keystream), strided Horner in r^LPF
    L5 R;
#pragma unroll
    for (int i = 0; i < 5; i++) R.v[i] = act ? Pp->rpow[C::LOG][i] : 0u;
    L5 acc = {{0, 0, 0, 0, 0}};
#pragma unroll
    for (int j = 0; j < C::ROWS; j++) {
      const uint32_t blk = sub + LPF * j;
      if (act && blk < nblk_ct) {
        const uint32_t q = blk;  // piece index within the page
        const uint4 k4 = *reinterpret_cast<const uint4*>(fl + (q >> 2) * kKsStride + (q & 3) * 16);
        const uint4 x = j < PPL ? ct[j < PPL ? j : 0] : make_uint4(0, 0, 0, 0);
        uint4 y = make_uint4(x.x ^ k4.x, x.y ^ k4.y, x.z ^ k4.z, x.w ^ k4.w);
        const uint32_t boff = blk * 16;
        if (boff + 16 > len) {  // tail: zero the bytes past the plaintext
          const uint32_t rem = len - boff;
          uint32_t yw[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
          for (int i = 0; i < 4; i++) {
            const uint32_t lo = 4 * i;
            const uint32_t keep = rem >= lo + 4 ? 0xffffffffu
                                  : (rem <= lo ? 0u : ((1u << (8 * (rem - lo))) - 1));
            yw[i] &= keep;
          }
          y = make_uint4(yw[0], yw[1], yw[2], yw[3]);
        }
        *reinterpret_cast<uint4*>(fl + boff) = y;
        acc = add5(mulmod(acc, R), block_limbs(x.x, x.y, x.z, x.w));
      } else if (act && blk == nblk_ct) {
        acc = add5(mulmod(acc, R), block_limbs(0u, 0u, len, 0u));  // le64(0) || le64(len)
      }
    }
    __builtin_amdgcn_wave_barrier();

    // 4) cross-lane tree inside the group: position p holds the lane whose last block has
    //    weight r^(LPF - p); level k multiplies by r^(2^k); finally * r.
    L5 v;
    {
      const int srcl = (int)(grp * LPF + ((sub + nb) & (LPF - 1)));
#pragma unroll
      for (int i = 0; i < 5; i++) v.v[i] = __shfl(acc.v[i], srcl);
    }
#pragma unroll
    for (int k = 0; k < C::LOG; k++) {
      L5 rk;
#pragma unroll
      for (int i = 0; i < 5; i++) rk.v[i] = act ? Pp->rpow[k][i] : 0u;
      L5 o;
#pragma unroll
      for (int i = 0; i < 5; i++) o.v[i] = __shfl_down(v.v[i], 1u << k);
      v = carry5(add5(mulmod(v, rk), o));
    }
    L5 r1;
#pragma unroll
    for (int i = 0; i < 5; i++) r1.v[i] = act ? Pp->rpow[0][i] : 0u;
    L5 tot = mulmod(v, r1);
#pragma unroll
    for (int i = 0; i < 5; i++) tot.v[i] = __shfl(tot.v[i], (int)(grp * LPF));
    bool ok = false;
    if (act) {
      const uint32_t sv[4] = {Pp->s[0], Pp->s[1], Pp->s[2], Pp->s[3]};
      uint32_t tag[4];
      poly_tag(tot, sv, tag);
      ok = ((tag[0] ^ Pp->tag[0]) | (tag[1] ^ Pp->tag[1]) | (tag[2] ^ Pp->tag[2]) |
            (tag[3] ^ Pp->tag[3])) == 0;
      if (!ok && sub == 0) {
        a.status[f] = CE_ERR_AUTH;
        atomicAdd(&a.counters[2], 1u);
        atomicMin(&a.counters[5], f);
      }
    }

    // 5) decode from LDS
    int32_t st = CE_OK;
    bool live = act && ok;
    if (live) {
      if (len < 16) st = CE_ERR_PT_LEN;
      else {
        const uint4 dv = *reinterpret_cast<const uint4*>(fl);
        bool found = false;
        for (uint32_t s = 0; s < a.n_supported; s++) {
          const uint4 sv = *reinterpret_cast<const uint4*>(a.supported + 16 * s);
          found |= dv.x == sv.x && dv.y == sv.y && dv.z == sv.z && dv.w == sv.w;
        }
        if (!found) st = CE_ERR_PT_VERSION;
      }
    }
    const uint8_t* body = fl + 16;
    const uint32_t blen = len >= 16 ? len - 16 : 0;
    uint64_t remaining = 0;
    uint32_t pos = 0;
    if (live && st == CE_OK) {
      Rd r{body, blen, 0};
      uint64_t count = 0;
      if (!rd_array_hdr(r, &count) || count > blen) st = CE_ERR_DECODE;
      else { remaining = count; pos = (uint32_t)r.i; }
    }
    const bool do_fold = live && st == CE_OK && (a.apply == nullptr || a.apply[f]);
    GroupFold gf{0xffffffffu, 0ull};
    for (;;) {
      const bool busy = live && st == CE_OK && remaining > 0;
      if (!__any(busy)) break;
      const uint32_t L = busy && pos + 34 <= blen ? dot_len_of_marker(body[pos + 33]) : 0u;
      bool valid = false;
      uint32_t k0 = 0, k1 = 0, k2 = 0, k3 = 0;
      unsigned long long ctr = 0;
      const uint32_t cand = pos + sub * L;
      if (L && sub < remaining && cand + L <= blen) {
        // 13 aligned LDS dwords -> the 48-byte window at cand
        const uint32_t* d = reinterpret_cast<const uint32_t*>(body) + (cand >> 2);
        const uint32_t sh = cand & 3;
        uint32_t dd[13];
#pragma unroll
        for (int i = 0; i < 13; i++) dd[i] = d[i];
        uint32_t w[12];
#pragma unroll
        for (int i = 0; i < 12; i++) w[i] = __builtin_amdgcn_alignbyte(dd[i + 1], dd[i], sh);
        valid = canon_dot(w, L, k0, k1, k2, k3, ctr);
      }
      constexpr unsigned long long GM = LPF == 64 ? ~0ull : ((1ull << LPF) - 1);
      const unsigned long long gb = (__ballot(valid) >> (grp * LPF)) & GM;
      const uint32_t k = gb == GM ? (uint32_t)LPF : (uint32_t)__builtin_ctzll(~gb);
      // general grammar for one element (group leader), e.g. reordered keys / array form
      const bool general = busy && k == 0;
      int gok = 0;
      uint32_t g0 = 0, g1 = 0, g2 = 0, g3 = 0, npos = pos;
      unsigned long long gc = 0;
      if (general && sub == 0) {
        Rd q{body, blen, pos};
        uint64_t aoff = 0, c = 0;
        gok = parse_dot(q, &aoff, &c);
        if (gok == 1) {
          g0 = ld_le32(body + aoff); g1 = ld_le32(body + aoff + 4);
          g2 = ld_le32(body + aoff + 8); g3 = ld_le32(body + aoff + 12);
          gc = c;
          npos = (uint32_t)q.i;
        }
      }
      gok = __shfl(gok, (int)(grp * LPF));
      npos = __shfl(npos, (int)(grp * LPF));
      if (general && gok != 1) st = CE_ERR_DECODE;
      const bool fold_fast = do_fold && busy && k > 0;
      const bool fold_gen = do_fold && general && gok == 1;
      if (__any(fold_fast || fold_gen)) {
        const bool active = (fold_fast && sub < k) || (fold_gen && sub == 0);
        fold_group<LPF>(a, f, active, fold_fast ? k0 : g0, fold_fast ? k1 : g1,
                        fold_fast ? k2 : g2, fold_fast ? k3 : g3, fold_fast ? ctr : gc, gf, grp,
                        sub);
      }
      if (busy && k > 0) {
        pos += k * L;
        remaining -= k;
      } else if (general && gok == 1) {
        pos = npos;
        remaining -= 1;
      }
    }
    if (gf.slot != 0xffffffffu && sub == 0) atomicMax(&a.batch[gf.slot], gf.best);
    if (live && st != CE_OK && sub == 0) {
      a.status[f] = st;
      atomicAdd(&a.counters[3], 1u);
      atomicMin(&a.counters[5], f);
    }
    __builtin_amdgcn_wave_barrier();
  }
}

hipError_t launch_open_fold_small(hipStream_t s, const DecodeArgs& a, int files_per_wave) {
  if (a.n == 0) return hipSuccess;
  const uint32_t groups = (a.n + files_per_wave - 1) / files_per_wave;
  // resident waves: LDS caps blocks per CU (160 KiB / block LDS)
  if (files_per_wave == 4) {
    const uint32_t blocks = std::min<uint32_t>((groups + 1) / 2, 256u * 4u);
    hipLaunchKernelGGL(k_open_fold_small<16>, dim3(blocks), dim3(128), 0, s, a);
  } else if (files_per_wave == 2) {
    const uint32_t blocks = std::min<uint32_t>((groups + 3) / 4, 256u * 4u);
    hipLaunchKernelGGL(k_open_fold_small<32>, dim3(blocks), dim3(256), 0, s, a);
  } else {
    const uint32_t blocks = std::min<uint32_t>((groups + 3) / 4, 256u * 8u);
    hipLaunchKernelGGL(k_open_fold_small<64>, dim3(blocks), dim3(256), 0, s, a);
  }
  return hipGetLastError();
}

// ----------------------------------------------------------------------------------------
// device version gate (crdt-enc/src/lib.rs:519-538) for batches in load_ops order
// ----------------------------------------------------------------------------------------
__global__ void k_gate_runs(GateArgs g) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.n) return;
  const uint32_t a = g.fa[i];
  if (a >= g.m) { atomicOr(&g.flags[0], 1u); return; }
  if (i == 0 || g.fa[i - 1] != a) {
    if (atomicAdd(&g.run_count[a], 1u) != 0) atomicOr(&g.flags[0], 1u);  // actor split
    g.run_first[a] = i;
  } else if (g.fv[i] != g.fv[i - 1] + 1) {
    atomicOr(&g.flags[0], 1u);  // versions not consecutive: host gate
  }
}

__global__ void k_gate_gap(GateArgs g) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.n) return;
  const uint32_t a = g.fa[i];
  if (a >= g.m) return;
  // consecutive run starting at version vf: a gap iff vf > expected (at the run's first file)
  if (g.run_first[a] == i && g.fv[i] > g.e0[a]) atomicMin(&g.flags[1], i);
}

__global__ void k_gate_apply(GateArgs g) {
  const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= g.n) return;
  const uint32_t a = g.fa[i];
  bool ap = false;
  if (a < g.m) {
    const uint64_t e0 = g.e0[a];
    const uint64_t vf = g.fv[g.run_first[a]];
    ap = g.fv[i] >= e0 && vf <= e0 && i < g.flags[1];
    if (ap) atomicMax(&g.newnov[a], (unsigned long long)(g.fv[i] + 1));
  }
  g.apply[i] = ap ? 1 : 0;
}

hipError_t launch_gate(hipStream_t s, const GateArgs& g) {
  if (g.n == 0) return hipSuccess;
  const uint32_t blocks = (g.n + 255) / 256;
  hipLaunchKernelGGL(k_gate_runs, dim3(blocks), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_gate_gap, dim3(blocks), dim3(256), 0, s, g);
  hipLaunchKernelGGL(k_gate_apply, dim3(blocks), dim3(256), 0, s, g);
  return hipGetLastError();
}

}  // namespace ce
