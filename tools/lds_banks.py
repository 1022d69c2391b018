"""LDS bank-conflict model of k_open_fold_v2's fast Dot decode (ce_fused.hip decode_fold).

Per ds_read_b32 the hardware serves lanes 0-31 and 32-63 as two groups, bank = (a / 4) mod 32
(MI355X_MICROARCH.md, LDS table); each extra distinct address on a bank within a group costs one
LDS cycle.  A wave holds 4 files (16 lanes each); lane `sub` reads the candidate Dots
done + sub (+ 16 on the second half of a round, skipped in a file's last round) as three aligned
runs: 3 dwords at c & ~3, 7 at (c + 9) & ~3, 3 at (c + 34) & ~3.  Prints, per region stride
(bytes between the wave's file regions in LDS), the mean extra cycles per read instruction and
group at the C2 layout (array header 3 B, 38-B Dots, 107 Dots) and averaged over Dot lengths
34..42 and header lengths 1 and 3.
  python3 tools/lds_banks.py"""
import collections


def cost(stride, ndots=107, L=38, pos=3):
    tot = extra = 0
    for done in range(0, ndots, 32):
        two = done + 16 < ndots
        for h in range(2 if two else 1):
            for off, nq in ((0, 3), (9, 7), (34, 3)):
                for q in range(nq):
                    for g in range(2):
                        banks = collections.defaultdict(set)
                        for lane in range(32):
                            f, sub = 2 * g + lane // 16, lane % 16
                            i = done + sub + 16 * h
                            cand = pos + i * L if (i < ndots and pos + i * L + L <= 4069) else 0
                            a = f * stride + 16 + ((cand + off) & ~3) + 4 * q
                            banks[(a // 4) % 32].add(a)
                        tot += 1
                        extra += max(len(v) for v in banks.values()) - 1
    return extra / tot


if __name__ == "__main__":
    print("stride  C2  mean(L 34..42, pos 1/3)")
    for s in range(4096, 4096 + 257, 16):
        vals = [cost(s, L=L, pos=pos) for pos in (1, 3) for L in (34, 35, 36, 38, 42)]
        print(s, round(cost(s), 3), round(sum(vals) / len(vals), 3))
