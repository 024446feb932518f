"""LDS bank-conflict check of the attention-image layouts of csrc/kernels/qkv_attn.hip.

Models the lane groups and bank widths of MI355X_MICROARCH.md §LDS for the three access
patterns of an image (128 rows x 128 B, 16-B chunk c of row r at slot swz(r, c)):
  * 16-B writes (ds_write_b128: 8 groups of 8 consecutive lanes, bank = dword mod 32):
    lane row G (16 lanes, fr = lane & 15) writes row (i + (G & 1))*16 + fr, chunk ch0 + (G >> 1)
  * fragment reads (ds_read_b128: 4 non-contiguous 16-lane groups, mod 64): row kt*16 + fr,
    chunk ds*4 + fc
  * transposed V reads (ds_read_b64_tr_b16: 2 x 32 lanes, mod 64): row ks*32 + fc*4 + (fr >> 2)
    (+16), chunk dt*2 + ((fr & 3) >> 1), 8-B half fr & 1
Prints the extra (conflict) cycles of the worst instruction of each pattern per swizzle.
"""


def conflicts(addr, groups, nbank, width):
    tot = 0
    for g in groups:
        banks = {}
        for lane in g:
            for w in range(width // 4):
                dw = addr[lane] // 4 + w
                banks.setdefault(dw % nbank, set()).add(dw)
        tot += max(len(v) for v in banks.values()) - 1
    return tot


G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[x + 32 for x in g] for g in G128]
G32 = [list(range(32)), list(range(32, 64))]
G8 = [list(range(k, k + 8)) for k in range(0, 64, 8)]


def check(swz):
    rd = max(conflicts([(kt * 16 + (l & 15)) * 128 + swz(kt * 16 + (l & 15), ds * 4 + (l >> 4)) * 16 for l in range(64)],
                       G128, 64, 16) for kt in range(8) for ds in range(2))
    tr = 0
    for ks in range(4):
        for c0 in range(0, 8, 2):
            for hi in (0, 16):
                ad = []
                for l in range(64):
                    fr, fc = l & 15, l >> 4
                    r = ks * 32 + fc * 4 + (fr >> 2) + hi
                    ad.append(r * 128 + swz(r, c0 + ((fr & 3) >> 1)) * 16 + (fr & 1) * 8)
                tr = max(tr, conflicts(ad, G32, 64, 8))
    wr = 0
    for i in range(0, 8, 2):
        for ch0 in range(0, 8, 2):
            ad = [((i + ((l >> 4) & 1)) * 16 + (l & 15)) * 128
                  + swz((i + ((l >> 4) & 1)) * 16 + (l & 15), ch0 + (l >> 5)) * 16 for l in range(64)]
            wr = max(wr, conflicts(ad, G8, 32, 16))
    return rd, tr, wr


if __name__ == "__main__":
    for name, f in (("c ^ (r & 7)  [qkv_attn images]", lambda r, c: c ^ (r & 7)),
                    ("c ^ ((r >> 1) & 7)  [GEMM operand images]", lambda r, c: c ^ ((r >> 1) & 7)),
                    ("c ^ (((r >> 1) & 3) << 1)  [attention.hip V]", lambda r, c: c ^ (((r >> 1) & 3) << 1))):
        rd, tr, wr = check(f)
        print(f"{name:45s} b128 reads +{rd}  tr16 reads +{tr}  b128 writes +{wr}")
