"""GPU unit test of the tile-pipeline setting of the wavefront launches (csrc/lif_layers.hip
snnflow_set_pipe / snnflow_get_pipe).  The forward pipeline itself is compared with the one-tile
bodies by test_gpu_parity.py::test_pipelined_slots_match_one_tile_slots; the backward runs one tile
per block only (its pipeline and a one-tile swapped-operand body measured no faster and were removed,
DESIGN.md round 5), so a backward tile count other than 0 is refused."""
import pytest

pytestmark = pytest.mark.gpu


def test_pipe_set_get():
    """snnflow_set_pipe / snnflow_get_pipe round trip; negative forward counts and backward counts
    other than 0 are refused and leave the setting unchanged."""
    from snnflow import _lib

    old = _lib.lib.snnflow_get_pipe(0)
    try:
        assert _lib.lib.snnflow_set_pipe(3, 0) == 0
        assert (_lib.lib.snnflow_get_pipe(0), _lib.lib.snnflow_get_pipe(1)) == (3, 0)
        assert _lib.lib.snnflow_set_pipe(-1, 0) != 0
        assert _lib.lib.snnflow_set_pipe(2, 1) != 0
        assert _lib.lib.snnflow_get_pipe(0) == 3
    finally:
        _lib.lib.snnflow_set_pipe(old, 0)
