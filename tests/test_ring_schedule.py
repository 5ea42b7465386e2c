"""CPU model of the scan kernels' LDS-DMA ring accounting.

Each kernel waits for a stage with a compile-time `s_waitcnt vmcnt(W)`: W is
the number of VMEM ops the wave issued AFTER the stage it needs.  A W that is
too large reads a stage before it lands (wrong keys); too small only costs
time.  Here the issue order of every kernel is replayed per wave and each
wait is checked to retire exactly the stages it must, for every stage count
per tile the kernels instantiate.

Formulas restated from fx_scan.hip (k_scan_v4).
"""
import pytest

NS = 5


def _stage(o):
    return o if isinstance(o, int) else o[1]


def _replay(spt, pieces, aux_first, pro_wait, loop_wait, tiles=4):
    """pieces: corpus VMEM ops per stage; aux_first: one extra op with the
    first stage of a tile.  The loop at stage g waits so that stage g+1 has
    landed and then issues stage g+NS-1."""
    ops = []

    def issue(st):
        ops.extend([st] * pieces)
        if aux_first and st % spt == 0:
            ops.append(("aux", st))

    for st in range(NS - 1):
        issue(st)
    w = pro_wait
    done, pend = ops[:len(ops) - w], ops[len(ops) - w:]
    assert all(_stage(o) > 0 for o in pend) and any(_stage(o) == 0 for o in done)
    for t in range(tiles):
        for j in range(spt):
            g = t * spt + j
            w = loop_wait(j)
            done, pend = ops[:len(ops) - w], ops[len(ops) - w:]
            assert all(_stage(o) > g + 1 for o in pend), (spt, g, w)
            assert any(_stage(o) == g + 1 for o in done), (spt, g, w)
            issue(g + NS - 1)


@pytest.mark.parametrize("ksteps", [8, 12, 16, 24])
def test_v4_waits(ksteps):
    spt = ksteps // 2
    # prologue: vmcnt(12); loop: W = 8 + ((j+3)%SPT==0) + ((j+2)%SPT==0)
    _replay(spt, 4, True, 12, lambda j: 8 + ((j + 3) % spt == 0) + ((j + 2) % spt == 0))
