"""Enumerate the LDS accesses of the GEMM/attention fragment reads and count bank conflicts.

Bank model (MI355X_MICROARCH.md §LDS): ds_read_b128 is serviced in four 16-lane
groups {0-3,12-15,20-27}, {4-11,16-19,28-31}, {32-35,44-47,52-59}, {36-43,48-51,60-63},
bank = (addr/4) % 64; ds_read_b64_tr_b16 / ds_read_b64 / ds_read_b32 in two 32-lane
halves (b32: bank = (addr/4) % 32).  A group costs max-over-banks(#distinct dwords).
Run: python tools/lds_bank_check.py  (prints the worst group cost per pattern; 1 = free)
"""

B128_GROUPS = [
    list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
    list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32)),
    list(range(32, 36)) + list(range(44, 48)) + list(range(52, 60)),
    list(range(36, 44)) + list(range(48, 52)) + list(range(60, 64)),
]
HALVES = [list(range(0, 32)), list(range(32, 64))]


def swz_k(row):
    return (row >> 1) & 7


def swz_mn(k):
    return 2 * (k & 3) + 8 * ((k >> 3) & 1)


def cost(addrs, groups, width, nbanks=64):
    worst = 0
    for grp in groups:
        banks = {}
        for lane in grp:
            for w in range(width // 4):
                dw = addrs[lane] // 4 + w
                banks.setdefault(dw % nbanks, set()).add(dw)
        # cycles for this group relative to its minimum
        need = max(len(v) for v in banks.values())
        worst = max(worst, need)
    return worst


def kmajor_b128(row0, kk):
    out = []
    for lane in range(64):
        row = row0 + (lane & 15)
        c = ((kk >> 3) + (lane >> 4)) ^ swz_k(row)
        out.append(row * 128 + c * 16)
    return out


def mnmajor_tr(R, row0, kk, i):
    RB = R * 2
    out = []
    for lane in range(64):
        t, g = lane & 15, lane >> 4
        q, p = t >> 2, t & 3
        chunk = (row0 >> 3) + (p >> 1)
        kr = kk + 8 * g + 4 * i + q
        out.append(kr * RB + (chunk ^ swz_mn(kr)) * 16 + (p & 1) * 8)
    return out


def mnmajor_f32(R, row0, kk, j):
    RB = R * 4
    out = []
    for lane in range(64):
        col, g = row0 + (lane & 15), lane >> 4
        cb = col * 4
        kr = kk + 8 * g + j
        out.append(kr * RB + (((cb >> 4) ^ swz_mn(kr)) << 4) + (cb & 15))
    return out


def main():
    w = max(cost(kmajor_b128(r0, kk), B128_GROUPS, 16) for r0 in range(0, 128, 16) for kk in (0, 32))
    print("k-major ds_read_b128 (bf16 frag) worst:", w)
    for R in (128, 256):
        w = max(cost(mnmajor_tr(R, r0, kk, i), HALVES, 8) for r0 in range(0, R, 16)
                for kk in (0, 32) for i in (0, 1))
        print(f"m/n-major ds_read_b64_tr_b16 R={R} worst:", w)
    for R in (128, 256):
        w = max(cost(mnmajor_f32(R, r0, 0, j), HALVES, 4, 32) for r0 in range(0, R, 16) for j in range(8))
        print(f"m/n-major f32 ds_read_b32 R={R} worst:", w)
    # the single-pass attention backward's dS^T tiles (csrc/attention.hip ds_off: [32 keys][32
    # queries] bf16, 64-B rows, 16-B chunk c of row r at c ^ ((r >> 2) & 3))
    w = max(cost(ds_tr32(k0, i), HALVES, 8) for k0 in (0, 16) for i in (0, 1))
    print("attention dS^T tile ds_read_b64_tr_b16 (phase 2) worst:", w)
    w = max(cost(ds_write(s_, hi), HALVES, 8) for s_ in (0, 1) for hi in (0, 1))
    print("attention dS^T tile ds_write_b64 (phase 1) worst:", w)


def ds_off(row, ch):
    return row * 64 + ((ch ^ ((row >> 2) & 3)) << 4)


def ds_tr32(k0, i):
    out = []
    for lane in range(64):
        g, tl = lane >> 4, lane & 15
        q, p = tl >> 2, tl & 3
        out.append(ds_off(k0 + 8 * i + 4 * (g >> 1) + q, 2 * (g & 1) + (p >> 1)) + ((p & 1) << 3))
    return out


def ds_write(s_, hi):
    # lane (key = lane & 31, h = lane >> 5) writes 8 B: chunk 2s (+1 for elements 4..7), half h
    return [ds_off(lane & 31, 2 * s_ + hi) + 8 * (lane >> 5) for lane in range(64)]


if __name__ == "__main__":
    main()
