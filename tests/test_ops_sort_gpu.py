"""``tmx::radix_sort`` (csrc/radix.hip, ops/sort.py) against ``torch.sort(..., stable=True)`` on the host: identical
indices (stability included) and bit-identical values for fp32 / fp64 / int32 / int64, ascending and descending,
ties, NaN, +-inf, signed zeros, 1-D and row-batched 2-D inputs, tile edges (4096 keys per tile), the one-workgroup row kernels' limits (4096;
16384 32-bit / 8192 64-bit keys)."""
import pytest
import torch

from torchmetrics_forked_amd import ops
from torchmetrics_forked_amd.ops.sort import sort

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _need_native(device):
    ops.require()


def _data(n, dtype, seed, rows=None):
    g = torch.Generator().manual_seed(seed)
    shape = (n,) if rows is None else (rows, n)
    if dtype.is_floating_point:
        x = (torch.randn(shape, generator=g, dtype=torch.float64) * 100).round() / 4  # many ties
        x = x.to(dtype)
        flat = x.view(-1)
        if flat.numel() > 20:
            flat[3::97] = float("nan")
            flat[5::89] = float("inf")
            flat[7::83] = float("-inf")
            flat[11::79] = -0.0
            flat[13::73] = 0.0
    else:
        x = torch.randint(-(1 << 20), 1 << 20, shape, generator=g, dtype=dtype)
        flat = x.view(-1)
        if flat.numel() > 20:
            flat[::5] = 7  # long tie run
            flat[1::101] = torch.iinfo(dtype).min
            flat[2::103] = torch.iinfo(dtype).max
    return x


def _native_sort(x, descending):
    """The radix kernel itself (every shape), not the routing wrapper ``ops.sort.sort``."""
    if x.dim() in (1, 2) and x.dtype in (torch.float32, torch.float64, torch.int32, torch.int64):
        v, i = torch.ops.tmx.radix_sort(x, descending)
        return v, i
    return sort(x, descending)


def _check(x, descending):
    v, i = _native_sort(x.cuda(), descending)
    ref = torch.sort(x, dim=-1, descending=descending, stable=True)
    assert i.dtype == torch.int64 and v.dtype == x.dtype
    assert torch.equal(i.cpu(), ref.indices)
    # bit-identical values (NaN payloads and signed zeros included)
    bits = torch.int64 if x.element_size() == 8 else torch.int32
    assert torch.equal(v.cpu().view(bits), ref.values.view(bits))


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
@pytest.mark.parametrize("n", [0, 1, 5, 4095, 4096, 4097, 8192, 8193, 12_345, 16_384, 16_385, 65_536, 100_003, 131_072, 131_073, 524_288, 524_289])
@pytest.mark.parametrize("descending", [False, True])
def test_radix_sort_matches_stable_torch_sort(dtype, n, descending):
    _check(_data(n, dtype, seed=n + 3), descending)


@pytest.mark.parametrize("dtype", [torch.float32, torch.int64])
def test_radix_sort_rows(dtype):
    _check(_data(9001, dtype, seed=1, rows=7), False)
    _check(_data(9001, dtype, seed=2, rows=7), True)
    _check(_data(8000, dtype, seed=3, rows=5), True)  # one 1024-thread workgroup per row (sort_block_kernel) for both


def test_radix_sort_large():
    _check(_data(3_000_017, torch.float32, seed=9), False)


def test_ranking_paths_use_native_sort():
    """Spearman / Kendall on the GPU (native sort + rank kernels) equal their host values."""
    from torchmetrics_forked_amd.functional.regression import kendall_rank_corrcoef, spearman_corrcoef

    g = torch.Generator().manual_seed(0)
    p = (torch.randn(20_000, generator=g) * 10).round()
    t = p * 0.5 + (torch.randn(20_000, generator=g) * 10).round()
    torch.testing.assert_close(spearman_corrcoef(p.cuda(), t.cuda()).cpu(), spearman_corrcoef(p, t), rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(kendall_rank_corrcoef(p.cuda(), t.cuda()).cpu(), kendall_rank_corrcoef(p, t), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("descending", [False, True])
def test_radix_sort_constant_digit_passes_skipped(descending):
    """>= 2^18 keys: digits equal in every key are not sorted on (labels in a small range, constants, rows)."""
    g = torch.Generator().manual_seed(5)
    _check(torch.randint(0, 1000, (300_001,), generator=g), descending)  # 2 of 8 int64 digits vary
    _check(torch.randint(-3, 3, (300_001,), generator=g, dtype=torch.int32), descending)  # sign flips every byte
    _check(torch.full((270_000,), 7, dtype=torch.int64), descending)  # every pass skipped: identity order
    _check(torch.full((270_000,), 0.5, dtype=torch.float32), descending)
    _check(torch.randint(0, 300, (4, 70_001), generator=g), descending)
    x = torch.rand(400_000, generator=g) * 0.25 + 0.5  # one exponent (float keys: every pass runs)
    _check(x, descending)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
@pytest.mark.parametrize("descending", [False, True])
def test_radix_sort_single_tile_rows(dtype, descending):
    """Rows of <= 4096 keys take the one-workgroup kernel (all passes in LDS, per-row constant digits skipped)."""
    _check(_data(4000, dtype, seed=21, rows=7), descending)
    _check(_data(1, dtype, seed=22, rows=3), descending)
    _check(_data(257, dtype, seed=23, rows=64), descending)
    const = torch.full((5, 300), 3, dtype=dtype)
    _check(const, descending)


@pytest.mark.parametrize("descending", [False, True])
def test_radix_sort_device_digit_plan(descending):
    """Integer rows beyond the one-launch sort (> 524,288 keys): the multi-launch passes take their digit skips from a
    plan decided on the device (no host read); skipped passes leave the buffers where they are."""
    g = torch.Generator().manual_seed(17)
    _check(torch.randint(0, 1000, (600_001,), generator=g), descending)  # 2 of 8 int64 digits vary
    _check(torch.randint(0, 70_000, (1_000_003,), generator=g, dtype=torch.int32), descending)  # 3 of 4: odd pass count
    _check(torch.full((700_000,), -5, dtype=torch.int64), descending)  # every pass skipped
    _check(torch.randint(-(1 << 40), 1 << 40, (800_000,), generator=g), descending)


def test_radix_sort_one_launch_opt_in():
    """TMX_SORT_COOP=1 (read once per process): 4096 < n <= 524,288 keys of one row in ONE cooperative launch with grid
    barriers -- exact against torch.sort at the tile-size edges, and one kernel for the whole sort."""
    import os
    import subprocess
    import sys

    code = (
        "import torch, sys; sys.path.insert(0, %r)\n"
        "from torchmetrics_forked_amd import ops; ops.require()\n"
        "sort = lambda x, d=False: torch.ops.tmx.radix_sort(x, d)\n"
        "g = torch.Generator().manual_seed(3)\n"
        "for n, dt in ((4097, torch.float32), (65_536, torch.float64), (131_073, torch.int64), (524_288, torch.float32)):\n"
        "    for desc in (False, True):\n"
        "        x = (torch.randn(n, generator=g, dtype=torch.float64) * 50).round().to(dt)\n"
        "        v, i = sort(x.cuda(), desc)\n"
        "        ref = torch.sort(x, descending=desc, stable=True)\n"
        "        assert torch.equal(i.cpu(), ref.indices) and torch.equal(v.cpu(), ref.values), (n, dt, desc)\n"
        "x = torch.randn(65536, device='cuda'); sort(x); torch.cuda.synchronize()\n"
        "from torch.profiler import profile, ProfilerActivity\n"
        "with profile(activities=[ProfilerActivity.CUDA]) as p:\n"
        "    sort(x); torch.cuda.synchronize()\n"
        "names = [e.name for e in p.events() if e.device_type.name == 'CUDA']\n"
        "k = [n for n in names if 'sort' in n.lower() or 'rs_' in n]\n"
        "print('KERNELS', len(k), k)\n"
    ) % os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    out = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=300,
                         env=dict(os.environ, TMX_SORT_COOP="1"))
    assert out.returncode == 0, out.stderr[-3000:]
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("KERNELS")][0]
    assert "sort_coop_kernel" in line and int(line.split()[1]) == 1, line


def test_sort_routing_picks_the_faster_engine():
    """``ops.sort.sort`` routes each shape class to the engine measured faster (``_faster_than_aten``) and returns the
    same stable order either way."""
    from torchmetrics_forked_amd.ops import sort as S

    cases = [(torch.randn(3, 9000), True), (torch.randn(4000), True), (torch.randn(8000), True), (torch.randn(8000, dtype=torch.float64), False),
             (torch.randn(70_000), False), (torch.randn(300_000), True),
             (torch.randn(70_000, dtype=torch.float64), False), (torch.randint(0, 9, (1 << 20,)), True)]
    for x, native in cases:
        assert S._faster_than_aten(x.cuda()) == native, (x.shape, x.dtype)
        v, i = sort(x.cuda())
        ref = torch.sort(x, stable=True)
        assert torch.equal(i.cpu(), ref.indices) and torch.equal(v.cpu(), ref.values)


@pytest.mark.parametrize("dtype", [torch.float32, torch.float64, torch.int32, torch.int64])
@pytest.mark.parametrize("descending", [False, True])
@pytest.mark.parametrize("kind", ["equal", "narrow", "two_values", "huge"])
def test_radix_sort_onesweep_edge_cases(dtype, descending, kind):
    """Round 6 one-sweep path (4096 < n <= 4M keys, one row): every key equal (no pass executes: identity order),
    keys with constant high digits (passes skipped on the device), two distinct values (one executed pass), and the
    largest routed size."""
    n = {"equal": 10_000, "narrow": 70_001, "two_values": 4_097, "huge": 1 << 22}[kind]
    g = torch.Generator().manual_seed(n)
    if kind == "equal":
        x = torch.full((n,), 3, dtype=dtype)
    elif kind == "narrow":
        x = torch.randint(0, 200, (n,), generator=g).to(dtype)
        if dtype.is_floating_point:
            x = x / 8 + 1.0  # few varying mantissa bits, constant exponent
    elif kind == "two_values":
        x = torch.randint(0, 2, (n,), generator=g).to(dtype)
    else:
        x = _data(n, dtype, 17)
    _check(x, descending)
