"""CPU checks of the halo-tiled 3x3 conv's layout decisions
(csrc/conv/conv3x3_halo.hip): the LDS chunk-swizzle table is bank-conflict-free
for every fragment start residue under the ds_read_b128 lane groups, the output
stage swizzle keeps a write's 4 rows on distinct 32-B spans, and the routing
predicate only takes the shapes the kernel was built for."""
import re
from pathlib import Path

from distributed_model_parallel_amd.ops import conv_igemm

SRC = Path(__file__).resolve().parents[1] / "csrc" / "conv" / "conv3x3_halo.hip"

# ds_read_b128 services 64 lanes in four 16-lane groups (MI355X_MICROARCH.md, LDS)
GROUPS = [[0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
          [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31]]
GROUPS += [[lane + 32 for lane in g] for g in GROUPS]


def _halo_key_table():
    src = SRC.read_text()
    m = re.search(r"halo_key\(int q\) \{ return \((0x[0-9a-fA-F]+)u >> \(4 \* \(q & 7\)\)\) & 7; \}", src)
    k = re.search(r"constexpr uint32_t kHaloKeys = (0x[0-9a-fA-F]+)u;", src)
    assert m and k, "halo_key / kHaloKeys definition changed: update this test"
    # the DMA side (halo_key) and the fragment reads (kHaloKeys) must agree
    assert int(m.group(1), 16) == int(k.group(1), 16)
    packed = int(m.group(1), 16)
    return [(packed >> (4 * i)) & 7 for i in range(8)]


def test_rotated_table_addressing_matches_key():
    # fragment reads: nibble (o & 7) of rotr(table, 4 * (q0 & 7)) ^ lh == key(q0 + o) ^ lh
    key = _halo_key_table()
    packed = sum(k << (4 * i) for i, k in enumerate(key))
    for q0 in range(64):
        r = 4 * (q0 & 7)
        rot = packed if r == 0 else ((packed >> r) | (packed << (32 - r))) & 0xFFFFFFFF
        for lh in range(4):
            kt = rot ^ (0x11111111 * lh)
            for o in range(3 * 58 + 3):
                for odd in (0, 1):
                    ch = ((kt >> (4 * (o & 7))) & 7) ^ (4 * odd)
                    assert ch == ((4 * odd + lh) ^ key[(q0 + o) & 7])


def test_halo_key_conflict_free_for_every_start_residue():
    key = _halo_key_table()
    for q0 in range(16):              # fragment start pixel (tap offsets make it arbitrary)
        for c0 in (0, 4):             # k-step half: chunks c0 + (lane >> 4)
            for g in GROUPS:
                slots = set()
                for lane in g:
                    q = q0 + (lane & 15)
                    c = c0 + (lane >> 4)
                    # 16-B bank slot within a 256-B window: pixel parity + swizzled chunk
                    slots.add(((q & 1) << 3) | (c ^ key[q & 7]))
                assert len(slots) == 16, (q0, c0, g)


def test_old_key_was_not_conflict_free():
    # the GEMM tiles' (q >> 1) & 7 key conflicts for unaligned starts (finding 28)
    bad = 0
    for q0 in range(16):
        for g in GROUPS:
            slots = {(((q0 + (lane & 15)) & 1) << 3) | ((lane >> 4) ^ (((q0 + (lane & 15)) >> 1) & 7))
                     for lane in g}
            bad += len(slots) < 16
    assert bad > 0


def test_stage_write_rows_on_distinct_spans():
    def stage_key(p):
        return ((p >> 2) & 3) << 1
    for base in range(0, 224, 16):
        for i in range(4):
            for chunk_pair in range(0, 8, 2):
                spans = set()
                for lh in range(4):
                    p = base + 4 * lh + i
                    # rows 4 apart share the 128-B half of the bank window; the
                    # swizzled chunk pair picks the 32-B span inside it
                    spans.add((chunk_pair ^ stage_key(p)) >> 1)
                assert len(spans) == 4


def test_routing_predicate():
    kind = conv_igemm._halo_kind
    assert kind(64, 64, 3, 3, 1, 1, 56, 56) == 64
    assert kind(64, 64, 3, 3, 2, 1, 56, 56) == 0      # strided
    assert kind(128, 128, 3, 3, 1, 1, 28, 28) == 128  # layer 2 (conv3x3_c128.hip)
    assert kind(128, 128, 3, 3, 1, 1, 30, 28) == 0    # c128 tiles are 4 whole rows
    assert kind(128, 128, 3, 3, 2, 1, 56, 56) == 0
    assert kind(64, 64, 3, 3, 1, 1, 16, 16) == 0      # other widths (kernels are built per W)
    assert kind(64, 128, 3, 3, 1, 1, 56, 56) == 0
    assert kind(64, 64, 1, 1, 1, 0, 56, 56) == 0
    assert kind(256, 256, 3, 3, 1, 1, 14, 14) == 0


C128 = Path(__file__).resolve().parents[1] / "csrc" / "conv" / "conv3x3_c128.hip"


def test_c128_key_conflict_free_for_every_start_residue():
    """conv3x3_c128.hip: 256-B halo pixels (one whole bank row each), key
    2 (q & 7) XOR-ed into the 16 chunks of a pixel.  Every ds_read_b128 service
    group hits 16 distinct 16-B slots for any fragment start and chunk base."""
    src = C128.read_text()
    assert "hkey(int q) { return (q & 7) << 1; }" in src, "hkey changed: update this test"

    def key(q):
        return (q & 7) << 1
    for q0 in range(16):
        for base in (0, 4, 8, 12):     # 8 wk + 4 (s & 1): the chunk base of a k-step
            for g in GROUPS:
                slots = {(base + (lane >> 4)) ^ key(q0 + (lane & 15)) for lane in g}
                assert len(slots) == 16, (q0, base, g)
    # the c64 period-8 table does not carry over to the 256-B pixel stride
    old = _halo_key_table()
    bad = sum(len({(lane >> 4) ^ old[(q0 + (lane & 15)) & 7] for lane in g}) < 16
              for q0 in range(16) for g in GROUPS)
    assert bad > 0
