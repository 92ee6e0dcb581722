"""CPU-only checks of the host side: the C-ABI library loads and exports every function that
include/iwq.h declares, struct layouts agree, host validation and error mapping behave like the
reference, and nothing silently falls back to the CPU."""
import ctypes
import os
import re

import numpy as np
import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def header_functions():
    src = open(os.path.join(ROOT, "include", "iwq.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(iwq_[a-z_0-9]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from iron_weight_only_quant_amd import _lib
    return _lib.load()


def test_library_exports_every_header_symbol(lib):
    from iron_weight_only_quant_amd import _lib
    names = header_functions()
    assert len(names) >= 9
    for n in names:
        assert hasattr(lib, n), n
    assert set(names) == set(_lib.EXPORTS)


def test_build_info_and_status_strings(lib):
    assert b"gfx950" in lib.iwq_build_info()
    assert lib.iwq_status_string(0) == b"ok"
    assert lib.iwq_status_string(3) == b"Invalid w_group_size"


def test_batch_entry_layout():
    from iron_weight_only_quant_amd._lib import IwqBatchEntry
    assert ctypes.sizeof(IwqBatchEntry) == 64


def test_workspace_bytes(lib):
    assert lib.iwq_workspace_bytes(4096, 4096, 128, 0) == 8 * 4096 * 32
    assert lib.iwq_workspace_bytes(4096, 4096, -1, 0) == 4096 * 16  # one-pass hand-off words + partial keys
    assert lib.iwq_workspace_bytes(100, 64, -2, 1) == 512
    assert lib.iwq_workspace_bytes(4096, 100, 128, 0) == 0  # invalid geometry


def test_host_validation_without_gpu(lib):
    """Argument validation happens on the host before any HIP call."""
    vp = ctypes.c_void_p
    call = lib.iwq_quantize_minmax
    dummy = vp(16)
    # bad group divisibility (AssertionError in the reference, quant_funcs.py:11)
    assert call(dummy, 8, 100, 100, 0, 4, 128, 0, 0, None, 100, None, None, None, None, 0, None, 0, None) == 2
    # invalid group mode (ValueError "Invalid w_group_size", quant_linear.py:906)
    assert call(dummy, 8, 128, 128, 0, 4, -3, 0, 0, None, 128, None, None, None, None, 0, None, 0, None) == 3
    # bad dtype / bits / shape
    assert call(dummy, 8, 128, 128, 7, 4, 128, 0, 0, None, 128, None, None, None, None, 0, None, 0, None) == 5
    assert call(dummy, 8, 128, 128, 0, 0, 128, 0, 0, None, 128, None, None, None, None, 0, None, 0, None) == 4
    assert call(dummy, 8, 128, 64, 0, 4, 128, 0, 0, None, 128, None, None, None, None, 0, None, 0, None) == 1
    # codes with n_bits > 8
    assert call(dummy, 8, 128, 128, 0, 9, 128, 0, 0, None, 128, dummy, None, None, None, 0, None, 0, None) == 7


def test_decode_entries_host_validation(lib):
    """iwq_tile_codes / iwq_w4a16_gemm / iwq_dequant_packed reject bad geometry on the host (no launch)."""
    from iron_weight_only_quant_amd import _lib as L
    vp = ctypes.c_void_p
    d = vp(4096)
    assert lib.iwq_tile_codes(None, 16, 128, d, None) == 9          # IWQ_ERR_ARG
    assert lib.iwq_tile_codes(d, 15, 128, d, None) == 1             # N % 16 (IWQ_ERR_SHAPE)
    assert lib.iwq_tile_codes(d, 16, 100, d, None) == 1             # K % 128
    assert lib.iwq_tile_codes(vp(4104), 16, 128, d, None) == 9      # 16-B alignment
    gemm = lib.iwq_w4a16_gemm
    # tile layout is a decode-only (M <= 16) format
    assert gemm(d, 17, 256, 256, d, d, d, 4, 128, 128, None, d, 128, L.IWQ_FLAG_TILED_CODES, None) == 9
    assert gemm(d, 1, 256, 256, d, d, d, 4, 128, 100, None, d, 100, 0, None) == 1      # N % 128
    assert gemm(d, 1, 256, 256, d, d, d, 4, 96, 128, None, d, 128, 0, None) == 2       # K % group
    assert gemm(d, 1, 256, 256, d, d, d, 5, 128, 128, None, d, 128, 0, None) == 4     # n_bits
    assert lib.iwq_dequant_packed(d, d, d, 4, 128, 128, 100, d, 100, None) != 0
    # NIB layout: a prefill-only (M >= 256) format; no variant / tile layout / generic path with it
    nibf = L.IWQ_FLAG_NIB_CODES
    assert gemm(d, 255, 256, 256, d, d, d, 4, 128, 256, None, d, 256, nibf, None) == 9
    assert gemm(d, 256, 256, 256, d, d, d, 4, 128, 256, None, d, 256, nibf | (75 << 16), None) == 9
    assert gemm(d, 256, 256, 256, d, d, d, 4, 128, 256, None, d, 256, nibf | L.IWQ_FLAG_TILED_CODES, None) == 9
    assert gemm(d, 256, 256, 256, d, d, d, 4, 128, 256, None, d, 256, nibf | L.IWQ_FLAG_FORCE_GENERIC, None) == 9
    assert gemm(d, 256, 256, 256, d, d, d, 4, 128, 128, None, d, 128, nibf, None) == 9   # N % 256
    assert gemm(d, 256, 256, 256, d, d, d, 4, 32, 256, None, d, 256, nibf, None) == 9    # g % 64
    assert lib.iwq_nib_codes(None, 16, 128, d, None) == 9          # IWQ_ERR_ARG
    assert lib.iwq_nib_codes(d, 16, 48, d, None) == 1              # K % 32 (IWQ_ERR_SHAPE)
    assert lib.iwq_nib_codes(d, 0, 128, d, None) == 1
    assert lib.iwq_nib_codes(d, 16, 128, vp(4100), None) == 9      # 16-B alignment


def test_batch_plan_host(lib):
    from iron_weight_only_quant_amd._lib import IwqBatchEntry
    t = (IwqBatchEntry * 3)()
    shapes = [(4096, 4096), (11008, 4096), (4096, 11008)]
    for i, (r, c) in enumerate(shapes):
        t[i].w = 4096 * (i + 1)
        t[i].out_deq = 4096 * (i + 10)
        t[i].rows, t[i].cols = r, c
    total = ctypes.c_int64()
    assert lib.iwq_batch_plan(t, 3, 0, 4, 128, ctypes.byref(total)) == 0
    units = [r * c // 512 for r, c in shapes]
    assert [t[i].unit_begin for i in range(3)] == [0, units[0], units[0] + units[1]]
    assert total.value == sum(units)
    t[1].cols = 4100
    assert lib.iwq_batch_plan(t, 3, 0, 4, 128, ctypes.byref(total)) == 2
    assert lib.iwq_batch_plan(t, 3, 0, 4, 96, ctypes.byref(total)) == 3


def test_no_cpu_fallback():
    from iron_weight_only_quant_amd.quant_funcs import pseudo_quantize_tensor
    from iron_weight_only_quant_amd.quant_linear import QuantLinear
    x = torch.randn(4, 128).half()
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        pseudo_quantize_tensor(x, n_bits=4, q_group_size=128)
    with pytest.raises(RuntimeError, match="ROCm GPU"):
        QuantLinear.from_linear(torch.nn.Linear(128, 4).half(), w_bit=4, w_group_size=128)


def test_quant_result_timeout_retry_logic():
    """QuantResult.has_nan on nan_flag bit 1 (an aborted per-tensor hand-off that wrote nothing,
    include/iwq.h): with a retry it re-runs once and reports the new flag; without one, or with bit 2
    (outputs invalid), it raises."""
    from iron_weight_only_quant_amd.kernels import QuantResult
    calls = []

    def retry(v):
        calls.append(v)
        return torch.tensor([v], dtype=torch.int32)
    r = QuantResult(None, None, None, None, torch.tensor([2], dtype=torch.int32), lambda: retry(0))
    assert not r.has_nan() and r.retried and calls == [0]
    assert not r.has_nan() and calls == [0]  # the retry runs once
    r = QuantResult(None, None, None, None, torch.tensor([3], dtype=torch.int32), lambda: retry(1))
    assert r.has_nan() and r.retried  # the re-run's own NaN bit
    r = QuantResult(None, None, None, None, torch.tensor([2], dtype=torch.int32), lambda: retry(2))
    with pytest.raises(RuntimeError, match="hand-off"):
        r.has_nan()  # the re-run aborted too
    r = QuantResult(None, None, None, None, torch.tensor([2], dtype=torch.int32))
    with pytest.raises(RuntimeError, match="hand-off"):
        r.has_nan()
    r = QuantResult(None, None, None, None, torch.tensor([4], dtype=torch.int32), lambda: retry(0))
    with pytest.raises(RuntimeError, match="invalid"):
        r.has_nan()  # a launch that went ahead without one workgroup: no retry can help
    assert not QuantResult(None, None, None, None, torch.tensor([0], dtype=torch.int32)).has_nan()


def test_geometry_errors_mirror_reference():
    from iron_weight_only_quant_amd.kernels import group_geometry
    assert group_geometry(4096, 11008, 128, 0) == (128, 4096 * 86)
    assert group_geometry(4096, 11008, -2, 0) == (11008, 4096)
    assert group_geometry(4096, 11008, -2, 1) == (4096, 11008)
    assert group_geometry(64, 32, -1, 1) == (2048, 1)
    with pytest.raises(AssertionError):
        group_geometry(100, 64, 128, 0)
    with pytest.raises(ValueError, match="Invalid w_group_size"):
        group_geometry(100, 64, 0, 0)


def test_quant_wrapper_noop_paths():
    from types import SimpleNamespace

    from iron_weight_only_quant_amd.quant_wrapper import quantize_model
    m = torch.nn.Sequential(torch.nn.Linear(8, 8))
    assert quantize_model(m, SimpleNamespace(w_bit=16, a_bit=16)) is m  # not weight-only
    assert isinstance(m[0], torch.nn.Linear)
    with pytest.raises(NotImplementedError):
        quantize_model(m, SimpleNamespace(w_bit=4, a_bit=16, w_group_size=128, w_symmetric=False, gptq=True),
                       verbose=False)


def test_synth_generator_properties():
    from oracle.synth import synth
    x = synth(0, (512, 512), "float16").astype(np.float32)
    assert abs(float(x.mean())) < 1e-3
    assert 0.018 < float(x.std()) < 0.025
    a = synth(5, (4, 1000), "float32")
    b = synth(5, (4, 1000), "float32")
    assert np.array_equal(a, b)
    # counter-based: any sub-range can be regenerated from its offset
    from oracle.synth import synth_f32
    assert np.array_equal(synth_f32(5, 1500, 100), a.reshape(-1)[1500:1600])


def test_packed_validation_on_host():
    """kernels._check_packed rejects codes/scales/zeros of the wrong size, dtype or device before
    any pointer reaches the C-ABI (no GPU needed: the check is pure host logic)."""
    from iron_weight_only_quant_amd.kernels import _check_packed
    dev = torch.device("cpu")
    N, K, g = 256, 512, 128
    codes = torch.zeros(N * K // 2, dtype=torch.uint8)
    s = torch.zeros(N * K // g, dtype=torch.float16)
    _check_packed("t", dev, codes, s, s, 4, g, N, K)
    _check_packed("t", dev, codes, torch.zeros(N, dtype=torch.float16), None, 4, -2, N, K)
    with pytest.raises(ValueError):
        _check_packed("t", dev, codes[:-1], s, s, 4, g, N, K)
    with pytest.raises(ValueError):
        _check_packed("t", dev, codes, s, s, 4, 64, N, K)
    with pytest.raises(TypeError):
        _check_packed("t", dev, codes, s.float(), None, 4, g, N, K)
    with pytest.raises(TypeError):
        _check_packed("t", dev, codes, s, s.bfloat16(), 4, g, N, K)
    with pytest.raises(ValueError):
        _check_packed("t", dev, codes, s, s, 8, g, N, K)
    with pytest.raises(ValueError):
        _check_packed("t", torch.device("cuda", 0), codes, s, s, 4, g, N, K)
    with pytest.raises(ValueError):
        _check_packed("t", dev, codes, s, s, 4, g, N, K, bias=torch.zeros(N + 1, dtype=torch.float16))


def test_tied_weight_detection():
    """quant_wrapper._tied: a layer whose weight bytes overlap an EARLIER layer's goes to the
    per-layer path; disjoint views of one buffer stay batchable."""
    from iron_weight_only_quant_amd.quant_wrapper import _tied
    a, b, c = torch.nn.Linear(8, 8), torch.nn.Linear(8, 8), torch.nn.Linear(8, 8)
    b.weight = a.weight
    assert _tied([("a", a), ("b", b), ("c", c)]) == {"b"}
    assert _tied([("b", b), ("a", a)]) == {"a"}
    big = torch.zeros(16, 8)
    d, e, f = torch.nn.Linear(8, 8), torch.nn.Linear(8, 8), torch.nn.Linear(8, 8)
    d.weight = torch.nn.Parameter(big[:8])
    e.weight = torch.nn.Parameter(big[8:])
    f.weight = torch.nn.Parameter(big[4:12])
    assert _tied([("d", d), ("e", e)]) == set()
    assert _tied([("f", f), ("d", d), ("e", e)]) == {"d", "e"}
    assert _tied([("d", d), ("e", e), ("f", f)]) == {"f"}


def _lint():
    import importlib.util
    spec = importlib.util.spec_from_file_location(
        "check_lds_waits", os.path.join(os.path.dirname(os.path.dirname(__file__)), "tools", "check_lds_waits.py"))
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def test_lds_wait_lint_model():
    """The lint's LDS-queue model: a use of an asm ds_read's registers before a wait that retires
    it is flagged; counted waits that retire it (writes queued behind it) are not."""
    L = _lint()
    ok = ["ds_read_b128 v[4:7], v1 offset:0", "ds_write_b128 v2, v[8:11] offset:0",
          "s_waitcnt lgkmcnt(1)", "v_mfma_f32_32x32x16_f16 a[0:15], v[4:7], v[12:15], a[0:15]"]
    assert L.check_kernel(ok) == []
    early = ["ds_read_b128 v[4:7], v1 offset:0", "ds_write_b128 v2, v[8:11] offset:0",
             "s_waitcnt lgkmcnt(2)", "v_lshrrev_b32_e32 v20, 8, v5"]
    assert len(L.check_kernel(early)) == 1
    # a write retired by the wait does not retire a read issued after it
    order = ["ds_write_b128 v2, v[8:11] offset:0", "ds_read_b128 v[4:7], v1 offset:0",
             "s_waitcnt lgkmcnt(1)", "v_mov_b32_e32 v30, v6"]
    assert len(L.check_kernel(order)) == 1


def test_store_hazard_lint_model():
    """The buffer-store data hazard: the instruction right after a 16-byte buffer store may not
    write that store's data registers (ROCm 7.2 LLVM omits the wait state with an SGPR soffset)."""
    L = _lint()
    bad = ["buffer_store_dwordx4 v[58:61], v2, s[8:11], s2 offen nt", "v_mov_b32_e32 v58, 0"]
    assert len(L.check_store_hazard(bad)) == 1
    ok = ["buffer_store_dwordx4 v[58:61], v2, s[8:11], s2 offen nt", "s_nop 0", "v_mov_b32_e32 v58, 0"]
    assert L.check_store_hazard(ok) == []
    reads = ["buffer_store_dwordx4 v[58:61], v2, s[8:11], s2 offen", "v_add_u32_e32 v3, v58, v2"]
    assert L.check_store_hazard(reads) == []


def test_lds_wait_lint_prefill_kernels():
    """Every hand-ordered prefill kernel (inline-asm LDS access, hand-counted lgkmcnt) as compiled
    for gfx950: no register of an LDS read is touched before its wait retires it."""
    if not os.path.exists("/opt/rocm/bin/hipcc"):
        pytest.skip("hipcc not available")
    L = _lint()
    import tempfile
    with tempfile.TemporaryDirectory() as d:
        out = os.path.join(d, "p.s")
        L.compile_asm(out)
        text = open(out).read()
    names = L.KERNELS.findall(text)
    assert len(names) >= 8
    for name in names:
        i = text.index(name + ":")
        assert L.check_kernel(text[i:text.index(".Lfunc_end", i)].split("\n")) == [], name


def test_host_abi_under_asan_ubsan():
    """SURVEY.md §5 sanitizers: the C-ABI's host code (batch plans, argument validation, kernel and
    split-K dispatch up to the launch) built from the library's own sources with host-side
    AddressSanitizer + UndefinedBehaviorSanitizer (tests/asan/Makefile, host-only objects) and driven
    by tests/asan/host_abi_check.c: every documented status, no sanitizer report (halt_on_error)."""
    import shutil
    import subprocess
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    if not os.path.exists("/opt/rocm/bin/hipcc") or shutil.which("make") is None:
        pytest.skip("hipcc / make not available")
    jobs = str(min(8, os.cpu_count() or 1))
    b = subprocess.run(["make", "-C", os.path.join(root, "tests", "asan"), "-j" + jobs], capture_output=True,
                       text=True, timeout=900)
    assert b.returncode == 0, b.stdout[-3000:] + b.stderr[-3000:]
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:halt_on_error=1:abort_on_error=0",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([os.path.join(root, "build", "asan", "host_abi_check")], capture_output=True, text=True,
                       timeout=300, env=env)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    assert "passed under ASan/UBSan" in r.stdout
    assert "runtime error" not in r.stderr and "AddressSanitizer" not in r.stderr


def test_quant_result_timeout_bit_raises():
    """include/iwq.h nan_flag bit 1 (the per-tensor one-pass hand-off aborted) is an error, not a NaN."""
    from iron_weight_only_quant_amd.kernels import QuantResult
    ok = QuantResult(None, None, None, None, torch.tensor([0], dtype=torch.int32))
    nan = QuantResult(None, None, None, None, torch.tensor([1], dtype=torch.int32))
    assert not ok.has_nan() and nan.has_nan()
    with pytest.raises(RuntimeError, match="hand-off"):
        QuantResult(None, None, None, None, torch.tensor([2], dtype=torch.int32)).has_nan()


def test_auto_fused_policy():
    """QuantLinear(fused_forward="auto")'s rule (kernels.auto_fused_preferred, profiles/
    r03_ab_auto_graph.jsonl, r05_ab_auto_g128.jsonl): per channel fused up to 192 rows (1024 on K >= 2N
    weights) and from 4096 rows on the LARGE_M_FUSED shapes; grouped up to 512 rows on K >= 2N, 128 on
    N > K, and on square weights up to 32 and from 96 to 192 rows; F.linear otherwise."""
    from iron_weight_only_quant_amd.kernels import auto_fused_preferred as P
    assert P(1, 11008, 4096, 128) and P(32, 4096, 4096, 128) and not P(64, 4096, 4096, 128)
    assert P(96, 4096, 4096, 128) and P(192, 4096, 4096, 128) and not P(255, 4096, 4096, 128)
    assert P(128, 11008, 4096, 128) and not P(192, 11008, 4096, 128)
    assert P(192, 11008, 4096, -2) and not P(193, 4096, 4096, -2) and not P(8192, 4096, 4096, -2)
    assert P(512, 4096, 11008, 128) and not P(1024, 4096, 11008, 128)
    assert P(1024, 4096, 11008, -2) and not P(2048, 4096, 11008, -2)
    # large M: the fused prefill only where it beats the library GEMM (kernels.LARGE_M_FUSED:
    # Llama-2-7B gate / up, per channel)
    assert P(8192, 11008, 4096, -2) and not P(2048, 11008, 4096, -2) and not P(8192, 11008, 4096, 128)
    assert not P(8192, 4096, 11008, -2) and not P(8192, 28672, 8192, -2)


def test_group_major_params_layout():
    """kernels.group_major_params: [N, K/g] reference order -> [K/g, N] (element g * N + n) for
    IWQ_FLAG_GROUP_MAJOR; zeros follow the scales, symmetric (None) stays None; per channel refused."""
    from iron_weight_only_quant_amd import kernels as K
    N, Kd, g = 256, 1024, 128
    s = torch.arange(N * Kd // g, dtype=torch.float32).half()
    z = (torch.arange(N * Kd // g) % 16).half()
    sg, zg = K.group_major_params(s, z, N, Kd, g)
    for n, gi in ((0, 0), (3, 5), (255, 7)):
        assert sg[gi * N + n] == s[n * (Kd // g) + gi] and zg[gi * N + n] == z[n * (Kd // g) + gi]
    assert sg.is_contiguous() and sg.numel() == s.numel()
    assert K.group_major_params(s, None, N, Kd, g)[1] is None
    with pytest.raises(ValueError):
        K.group_major_params(s, z, N, Kd, -2)


def test_trace_sections_cuts_a_kernel_trace_into_bench_regions(tmp_path):
    """tools/trace_sections.py (round 5): dispatches are assigned to bench.py --mark-file regions by the
    host clock that makes every region non-empty, same-name regions (the rounds of one interleaved arm)
    merge, and the dominant kernel's average is set beside bench.py's own per-call figure."""
    import csv
    import json
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools"))
    import trace_sections as TS
    d = tmp_path / "prof"
    d.mkdir()
    rows = []
    # region A: 4 launches of 10 us at t = 1000.., region B (two rounds): 2 x 3 launches of 5 us + a small
    # kernel, a dispatch outside every region
    for i in range(4):
        rows.append(("k_big", 1_000_000 + i * 11_000, 1_000_000 + i * 11_000 + 10_000))
    for base in (2_000_000, 3_000_000):
        for i in range(3):
            rows.append(("k_mid", base + i * 6_000, base + i * 6_000 + 5_000))
        rows.append(("k_tiny", base + 20_000, base + 20_500))
    rows.append(("k_outside", 5_000_000, 5_001_000))
    with open(d / "run_kernel_trace.csv", "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Kernel_Name", "Start_Timestamp", "End_Timestamp"])
        for n, s, e in rows:
            w.writerow([n, s, e])
    off = 777  # the "mono" clock is shifted: only "boot" puts every dispatch inside its region
    marks = [{"region": "A", "t0": {"boot": 990_000, "mono": 990_000 + off, "real": 0},
              "t1": {"boot": 1_050_000, "mono": 1_050_000 + off, "real": 1}, "bench_kernel_ms": 0.0100},
             {"region": "B", "t0": {"boot": 1_990_000, "mono": 9e18, "real": 0},
              "t1": {"boot": 2_030_000, "mono": 9e18, "real": 1}, "bench_ms_per_call_this_round": 0.0050},
             {"region": "B", "t0": {"boot": 2_990_000, "mono": 9e18, "real": 0},
              "t1": {"boot": 3_030_000, "mono": 9e18, "real": 1}, "bench_ms_per_call_this_round": 0.0052}]
    (tmp_path / "marks.jsonl").write_text("".join(json.dumps(m) + "\n" for m in marks))
    res = TS.summarize(TS.load_trace(str(d)), TS.load_marks(str(tmp_path / "marks.jsonl")))
    assert res["clock"] == "boot" and res["regions_with_dispatches"] == 3
    a, b = res["rows"]
    assert a["region"] == "A" and [k["kernel"] for k in a["kernels"]] == ["k_big"]
    assert a["kernels"][0]["dispatches"] == 4 and a["kernels"][0]["avg_us"] == 10.0
    assert a["kernels"][0]["median_gap_us"] == 1.0 and a["dominant_avg_over_bench"] == 1.0
    assert b["region"] == "B" and b["kernels"][0]["kernel"] == "k_mid" and b["kernels"][0]["dispatches"] == 6
    assert b["kernels"][1]["kernel"] == "k_tiny" and b["kernels"][1]["dispatches"] == 2
    assert b["bench"]["bench_ms_per_call_this_round"] == 0.0051  # median over the merged rounds
    assert abs(b["dominant_avg_over_bench"] - 5.0 / 5.1) < 1e-3


def test_e2m1_closed_form():
    """csrc/iwq_fp.hip e2m1_mag2: the E2M1 FP codec's encode-then-decode magnitude in closed form (the
    table-free pack path) equals the reference's _float_to_fp / _fp_to_float (quant_linear.py:126-163,
    213-235) on every fp16 magnitude the kernel can see (|t| clamped to fp_max = 6.0), per the
    exhaustive fixtures tests/golden/make_golden.py wrote by importing the reference.  This restates
    the kernel's packed 16-bit arithmetic lane by lane."""
    d = np.load(os.path.join(ROOT, "tests", "golden", "fp_small.npz"))
    x, enc, dec = d["in/all_fp16"], d["enc/e2m1"], d["dec/e2m1"]
    a = x.view(np.uint16).astype(np.int64) & 0x7FFF
    ref = np.abs(dec[enc].astype(np.float16)).view(np.uint16).astype(np.int64)
    dom = a <= 0x4600
    assert dom.sum() > 35000
    mt = ((a & 0x3FF) + 0x7EFF) & 0xFFFF
    nb = (a & 0x7C00) | ((mt & 0x8000) >> 6)
    ge1 = np.where(((a + 0x4400) & 0x8000) != 0, 0xFFFF, 0)
    gtq = np.where(((a + 0x4BFF) & 0x8000) != 0, 0xFFFF, 0)
    got = np.maximum(nb & ge1, gtq & 0x3800)
    assert np.array_equal(got[dom], ref[dom])


def test_bench_summary_is_last_and_compact():
    """bench.py's record ends with `summary` (the driver keeps only the stdout tail): the headline
    roofline figures, every section's key fraction, a few hundred bytes; missing sections are skipped."""
    import importlib.util
    import json
    spec = importlib.util.spec_from_file_location(
        "bench_for_summary", os.path.join(os.path.dirname(os.path.dirname(__file__)), "bench.py"))
    b = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(b)
    rec = {"roofline": {"frac": 0.76, "kernel_over_ceiling": 0.99, "fresh_ceiling": {"GBps": 6200.0},
                        "kernel_over_fresh_ceiling": 0.98, "other_placement": {"placement": "in-place", "frac": 0.74},
                        "traffic": 2.0e9, "alg_bytes_per_launch": 1.0e9},
           "shapes": {"4096x4096": {"frac": 0.61, "frac_beyond_launch_floor": 0.71}},
           "fused_forward": {"rows": [{"shape": "q_proj", "weights": "per-channel", "M": 1, "fused_vs_F_linear": 3.1}]},
           "formats": {"rows": [{"path": "fp4_e2m1_g128_asym_pack", "frac_of_hbm_peak": 0.67}]},
           "llama2_70b": {"roofline": {"frac": 0.74}}, "cpu_baseline": {"value": 0.45}}
    s = b.summary_of(rec)
    assert s["frac"] == 0.76 and s["traffic_over_alg"] == 2.0 and s["other_placement"] == ["in-place", 0.74]
    assert s["shapes_frac"]["4096x4096"] == [0.61, 0.71]
    assert s["fused_vs_F_linear"]["q_proj/pc/M1"] == 3.1
    assert s["formats_frac"]["fp4_e2m1_g128_asym_pack"] == 0.67 and s["llama2_70b_frac"] == 0.74
    assert len(json.dumps(s)) < 2000
    assert set(b.summary_of({"roofline": {"frac": 0.7}})) >= {"frac"}  # sections absent (N > 1 runs)
