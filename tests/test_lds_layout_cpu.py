"""Bank-conflict model of the conv epilogue's LDS layouts (csrc/conv_gemm.hip), on the gfx950 LDS
rules of MI355X_MICROARCH.md ("LDS [CDNA4]": lane groups per instruction, bank = (a/4) mod 32 for
stores and mod 64 for b64 / b128 reads; identical addresses broadcast).

The C tile of a 16-bit FWD / DGRAD epilogue with BN <= 128 is staged in 8-byte pieces XOR-swizzled
by a 4-bit row function and read back as two ds_read_b64 per 16-byte chunk; the previous 16-byte
chunk layout put two lanes of every ds_write_b64 group on one bank pair (profiles/pmc_r5_step.md:
17-35 % conflicts on the layer-1 launches; profiles/ab_r6.md section 9: 0.0 % now). These tests
pin the formulas -- a change to the swizzle that reintroduces conflicts fails here on the CPU."""
from collections import defaultdict

import pytest

WRITE_B64_GROUPS = [list(range(g * 16, g * 16 + 16)) for g in range(4)]
READ_B64_GROUPS = [list(range(0, 32)), list(range(32, 64))]
READ_B128_GROUPS = [
    [0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
    list(range(4, 12)) + [16, 17, 18, 19, 28, 29, 30, 31],
    [32, 33, 34, 35, 44, 45, 46, 47] + list(range(52, 60)),
    list(range(36, 44)) + [48, 49, 50, 51, 60, 61, 62, 63],
]


def extra_cycles(groups, lane_addrs, nbanks):
    """Sum over lane groups of (max distinct dword addresses on one bank - 1)."""
    extra = 0
    for grp in groups:
        per_bank = defaultdict(set)
        for lane in grp:
            for a in lane_addrs[lane]:
                per_bank[(a // 4) % nbanks].add(a)
        extra += max(len(v) for v in per_bank.values()) - 1
    return extra


def dwords(addr, nbytes):
    return [addr + 4 * k for k in range(nbytes // 4)]


def cswz(row, BN):
    if BN == 64:
        return (row & 12) | ((row & 1) << 1) | ((row >> 1) & 1)
    return row & 15


def piece_write_addr(row, col, BN):
    return row * (BN * 2) + ((((col >> 2) ^ cswz(row, BN))) << 3)


def chunk_write_addr(row, col, BN):   # the round-5 16-byte chunk layout
    CPR = BN // 8
    return row * (BN * 2) + (((col >> 3) ^ (row & (CPR - 1))) << 4) + ((col & 4) << 1)


def write_pattern(BN, addr_fn, WM=2, WN=2, BM=128):
    """Every ds_write_b64 of the C-tile staging: lane l holds row wr*(BM/WM) + i*16 + (l&15),
    columns wc*(BN/WN) + j*16 + 4*(l>>4) .. +3 (MFMA with swapped operands)."""
    MI, NI = BM // WM // 16, BN // WN // 16
    total = 0
    for wr in range(WM):
        for wc in range(WN):
            for i in range(MI):
                for j in range(NI):
                    lanes = {}
                    for l in range(64):
                        row = wr * (BM // WM) + i * 16 + (l & 15)
                        col = wc * (BN // WN) + j * 16 + 4 * (l >> 4)
                        lanes[l] = dwords(addr_fn(row, col, BN), 8)
                    total += extra_cycles(WRITE_B64_GROUPS, lanes, 32)
    return total


@pytest.mark.parametrize("BN", [64, 128])
def test_piece_layout_c_tile_writes_conflict_free(BN):
    assert write_pattern(BN, piece_write_addr) == 0


@pytest.mark.parametrize("BN", [64, 128])
def test_chunk_layout_had_write_conflicts(BN):
    # documents what the piece layout fixed: 2-way on every write group
    assert write_pattern(BN, chunk_write_addr) > 0


@pytest.mark.parametrize("BN,NTH", [(64, 256), (128, 256), (128, 512)])
def test_piece_layout_reader_conflict_free(BN, NTH):
    """Reader thread t: chunk cc = t % CPR of rows rg + RG*k (rg = t / CPR); two ds_read_b64 at
    piece 2cc and 2cc+1 (the second address = the first ^ 8)."""
    CPR = BN // 8
    RG = NTH // CPR
    for wave in range(NTH // 64):
        for k in range(4):
            for half in range(2):
                lanes = {}
                for l in range(64):
                    t = wave * 64 + l
                    cc, rg = t % CPR, t // CPR
                    row = rg + RG * k
                    a = row * (BN * 2) + (((2 * cc) ^ cswz(row, BN)) << 3)
                    lanes[l] = dwords(a ^ (8 * half), 8)
                assert extra_cycles(READ_B64_GROUPS, lanes, 64) == 0, (BN, NTH, wave, k, half)


@pytest.mark.parametrize("BN", [64, 128])
def test_piece_layout_is_a_permutation_of_each_row(BN):
    for row in range(64):
        slots = {piece_write_addr(row, col, BN) for col in range(0, BN, 4)}
        assert slots == {row * BN * 2 + 8 * p for p in range(BN // 4)}


def test_row_tile_fragment_reads_conflict_free_at_any_row_offset():
    """frag_row / the HALO slab: 128-B rows, 16-B chunk c at (c ^ (row & 7)); ds_read_b128 of rows
    d + (l & 15), chunk s*4 + (l >> 4) -- conflict-free for every row offset d (taps shift it)."""
    for d in range(16):
        for s in range(2):
            lanes = {}
            for l in range(64):
                row = d + (l & 15)
                chunk = s * 4 + (l >> 4)
                lanes[l] = dwords(row * 128 + ((chunk ^ (row & 7)) << 4), 16)
            assert extra_cycles(READ_B128_GROUPS, lanes, 64) == 0, (d, s)


def test_statistics_reduction_writes_conflict_free():
    """The epilogue's per-row-group partial sums (EPO = 8): column pair k of chunk cc at slot
    (k + cc/4 + 2*(rg&1)) & 3 -- every ds_write_b64 group of 16 lanes covers all 32 banks."""
    def spos(cc, k, g):
        return cc * 8 + 2 * ((k + (cc >> 2) + 2 * (g & 1)) & 3)
    for BN, NTH in ((128, 256), (64, 256), (128, 512)):
        CPR = BN // 8
        for wave in range(NTH // 64):
            for k in range(4):
                lanes = {}
                for l in range(64):
                    t = wave * 64 + l
                    cc, rg = t % CPR, t // CPR
                    lanes[l] = dwords(4 * (rg * BN + spos(cc, k, rg)), 8)
                assert extra_cycles(WRITE_B64_GROUPS, lanes, 32) == 0, (BN, NTH, wave, k)
