"""CPU: the uniform kernel's tile map (gcm_kernels.hip, QGCM_TILE_POOL 4) covers every tile of a launch
exactly once.  A restatement of the kernel's index arithmetic: workgroup g's LDS pool index i names tile
g*16 + i%16 + (i/16)*grid*16 while i < sidx (its share of the launch's first full rows), and the shared
tail hands out tiles tail0, tail0 + 1, ... up to ntiles; without a full row (or without a pool set) every
workgroup takes its mode-1 tiles up to ntiles.  The GPU tests (tests/test_gpu_tail_pool.py) check the
bytes; this checks the partition for many grid and batch shapes, including ragged last rows."""
import pytest

KW = 16  # waves (tiles in flight) per workgroup


def tail_split(ntiles, grid, eighths=4, pool=True):
    rows = ntiles // (grid * KW)
    if not pool or rows == 0:
        return None, None
    tail_rows = 0 if rows < 2 else min(rows - 1, max(1, rows * eighths // 8))
    return (rows - tail_rows) * KW, (rows - tail_rows) * grid * KW


def tiles_of_launch(ntiles, grid, eighths=4, pool=True):
    sidx, tail0 = tail_split(ntiles, grid, eighths, pool)
    got = []
    for g in range(grid):
        i = 0
        while True:
            if sidx is not None and i >= sidx:
                break
            t = g * KW + (i % KW) + (i // KW) * grid * KW
            if t >= ntiles:
                break
            got.append(t)
            i += 1
    if sidx is not None:
        got.extend(range(tail0, ntiles))
    return got


@pytest.mark.parametrize("grid", [1, 7, 512])
@pytest.mark.parametrize("eighths", [1, 4, 6, 8])
@pytest.mark.parametrize("rows,extra", [(0, 5), (1, 0), (1, 33), (2, 0), (2, 1), (3, 100), (8, 0), (9, 511)])
def test_every_tile_exactly_once(grid, eighths, rows, extra):
    ntiles = rows * grid * KW + extra
    got = tiles_of_launch(ntiles, grid, eighths)
    assert sorted(got) == list(range(ntiles))


def test_tail_share_of_the_headline_launch():
    # 2^20 packets = 65536 tiles on 256 CUs x 2 workgroups: 8 rows, the last 4 shared
    sidx, tail0 = tail_split(65536, 512)
    assert (sidx, tail0) == (4 * KW, 32768)


def test_without_pool_every_tile_is_static():
    assert sorted(tiles_of_launch(5 * 512 * KW + 77, 512, pool=False)) == list(range(5 * 512 * KW + 77))
