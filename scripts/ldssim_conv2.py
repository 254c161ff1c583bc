#!/usr/bin/env python3
"""LDS bank-conflict model of the fp32 conv2 kernels' A-operand reads (ds_read_b128).

A wave64 ds_read_b128 is serviced in four 16-lane groups (lanes {0-3,12-15,20-27}, {4-11,16-19,28-31}
and the same +32); within a group each extra distinct address on a 4-byte bank ((byte address / 4)
mod 64) costs one more LDS cycle (cdna_hip_programming.md section 2, MI355X_MICROARCH.md, LDS).
This walks every tile of a B = 100 launch and every tap, builds the 64 lane addresses the kernel
issues, and reports LDS cycles per group relative to the conflict-free 1.0:

    python scripts/ldssim_conv2.py [--search]

conv2_fwd (f32_fwd.hip): tile = 4 pooling windows x 2x2 pixels on the MFMA row axis (lane lr),
4-channel chunk 4 lg of 16 c2: address ((18 b + y - R0) RW + x) PS + 16 c2 + 4 lg.
conv2_bwd dgrad (f32_bwd.hip): tile = 16 consecutive output pixels; address of the routed gradient
(padded row, padded col) x PS + 16 cq + 4 lg in a 18-column tall image.
"""
import argparse

G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 += [[lane + 32 for lane in g] for g in G128]


def cycles(addrs):
    tot = 0
    for g in G128:
        banks = {}
        for lane in g:
            a = addrs[lane]
            for k in range(4):
                banks.setdefault((a + k) % 64, set()).add(a + k)
        tot += max(len(v) for v in banks.values())
    return tot


def conv2_fwd(PS, RW, B=100, TPB=5, stride=7):
    nwin = 49 * B
    tot = ideal = 0
    for blk in range(0, (nwin // 4 + TPB - 1) // TPB, stride):
        T0 = blk * TPB
        gw0 = 4 * T0
        b0 = gw0 // 49
        R0 = 18 * b0 + 2 * ((gw0 - 49 * b0) // 7)
        for i in range(TPB):
            for kh in range(5):
                for kw in range(5):
                    for c2 in range(2):
                        addrs = []
                        for lane in range(64):
                            lr, lg = lane & 15, lane >> 4
                            m = 16 * (T0 + i) + lr
                            gw = min(m >> 2, nwin - 1)
                            d = m & 3
                            bb, win = gw // 49, gw % 49
                            py, px = win // 7, win % 7
                            y, x = 2 * py + (d >> 1) + kh, 2 * px + (d & 1) + kw
                            addrs.append(((18 * bb + y - R0) * RW + x) * PS + 16 * c2 + 4 * lg)
                        tot += cycles(addrs)
                        ideal += 4
    return tot / ideal


def conv2_fwd8(PS=32, RW=18, B=100, TPB=5, stride=7, swizzle=True):
    """The 8-wave conv2_fwd layout (f32_fwd.hip, f32_conv2_fwd8_kernel): unpadded pixels, the 16-byte
    chunk c of pixel (row r, column x) stored at c ^ 2 ((r + x) & 3)."""
    nwin = 49 * B
    tot = ideal = 0
    for blk in range(0, (nwin // 4 + TPB - 1) // TPB, stride):
        T0 = blk * TPB
        gw0 = 4 * T0
        b0 = gw0 // 49
        R0 = 18 * b0 + 2 * ((gw0 - 49 * b0) // 7)
        for i in range(TPB):
            for kh in range(5):
                for kw in range(5):
                    for c2 in range(2):
                        addrs = []
                        for lane in range(64):
                            lr, lg = lane & 15, lane >> 4
                            m = 16 * (T0 + i) + lr
                            gw = min(m >> 2, nwin - 1)
                            d = m & 3
                            bb, win = gw // 49, gw % 49
                            py, px = win // 7, win % 7
                            r = 18 * bb + 2 * py + (d >> 1) + kh - R0
                            x = 2 * px + (d & 1) + kw
                            ch = (4 * c2 + lg) ^ ((2 * ((r + x) & 3)) if swizzle else 0)
                            addrs.append((r * RW + x) * PS + 4 * ch)
                        tot += cycles(addrs)
                        ideal += 4
    return tot / ideal


def conv2_bwd_dgrad(PS, B=100, TPB=10, stride=5):
    np_ = 196 * B
    tot = ideal = 0
    for blk in range(0, (np_ // 16 + TPB - 1) // TPB, stride):
        T0 = blk * TPB
        P0 = 16 * T0
        b0 = P0 // 196
        R0 = 18 * b0 + (P0 - 196 * b0) // 14
        for cq in range(4):
            for i in range(TPB):
                addrs = []
                for lane in range(64):
                    lr, lg = lane & 15, lane >> 4
                    P = min(16 * (T0 + i) + lr, np_ - 1)
                    bb, p = P // 196, P % 196
                    py, px = p // 14, p % 14
                    addrs.append(((18 * bb + py - R0) * 18 + px) * PS + 16 * cq + 4 * lg)
                tot += cycles(addrs)
                ideal += 4
    return tot / ideal


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--search", action="store_true", help="scan pixel strides / row lengths")
    a = ap.parse_args()
    print(f"conv2_fwd  PS 40 RW 20 (current): {conv2_fwd(40, 20):.2f}   PS 36 RW 24 (round 3): {conv2_fwd(36, 24):.2f}")
    print(f"conv2_fwd 8-wave form, PS 32 RW 18, chunks XOR 2((row + col) & 3): {conv2_fwd8():.2f} "
          f"(unswizzled: {conv2_fwd8(swizzle=False):.2f})")
    print(f"conv2_bwd dgrad PS 68, 18-pixel rows (round 3; now 72 x 22: conflict-free): {conv2_bwd_dgrad(68):.2f}")
    if a.search:
        for PS in (32, 36, 40, 44, 48):
            print("conv2_fwd PS", PS, " ".join(f"RW{RW}:{conv2_fwd(PS, RW, stride=28):.2f}" for RW in (18, 20, 22, 24, 26)))
        print("conv2_bwd dgrad", " ".join(f"PS{PS}:{conv2_bwd_dgrad(PS, stride=20):.2f}" for PS in range(64, 136, 4)))


if __name__ == "__main__":
    main()
