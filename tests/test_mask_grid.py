"""The persistent-grid rule for a CU-masked stream (nstl_mask_grid, the host
function behind nstl_stream_cus): mask bit i is a CU of XCD i % 8, shader engine
(i / 8) % 4 (tools/micro/cu_probe.hip, profiles/r4_cu_probe.txt); workgroups are
dealt round-robin over the XCDs and their SEs, so a one-per-CU grid is 32 x the
fewest CUs left on any (XCD, SE) pair.  Host-only: runs without a GPU."""
import pytest

from neurosync_trainer_lite_amd import _hip as K


@pytest.mark.parametrize("excluded,grid", [
    (set(), 256),
    ({0}, 224),                          # one CU: its SE's share sets the grid
    (set(range(8)), 224),                # one per XCD, all on SE 0
    (set(range(32)), 224),               # one per (XCD, SE): the smallest balanced cession
    (set(range(64)), 192),
    ({0, 8}, 224),                       # XCD 0, SEs 0 and 1
    ({0, 32}, 192),                      # two CUs of XCD 0's SE 0
    (set(range(0, 256, 8)), 0),          # every CU of XCD 0: no grid (nstl_stream_cus keeps all CUs)
])
def test_mask_grid(excluded, grid):
    assert K.mask_grid(excluded) == grid


def test_mask_grid_rejects_odd_sizes():
    assert K.mask_grid(set(), ncu=200) == 0
