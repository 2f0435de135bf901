"""Same-box A/B of the hand-written GEMMs against the vendor library (hipBLASLt through torch.mm).

Not a product path: the framework has one GEMM backend (ops.linear -> gfx950 MFMA kernels). This tool
patches ``ops.linear`` / ``ops.linear_rope_kv`` so prefill / encoder GEMMs (M > 64, no residual) run on
hipBLASLt plus the framework's epilogue kernels, then runs ``bench.py`` with the given arguments - the
"library" arm of profiles/r2/policy_ab*/. ``--tuned`` first loads the TunableOp solution table measured
on MI355X (tools/data/tunableop_mi355x.csv, lookup only).

    python tools/blas_ab.py [--tuned] -- --steps 4 --warmup 2 --no-probes --json-out gpurun_out/blas.json
"""
from __future__ import annotations

import os
import runpy
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from generativeaiexamples_amd import ops  # noqa: E402


def blas_linear(x2, w, bias, act, out_dtype):
    """hipBLASLt GEMM + the framework's own elementwise epilogue kernel."""
    y = torch.addmm(bias, x2, w.t()) if bias is not None else torch.mm(x2, w.t())
    if act == "swiglu":
        z = torch.empty(y.shape[0], y.shape[1] // 2, dtype=y.dtype, device=y.device)
        ops.native().silu_mul_interleaved(y, z)
        y = z
    elif act == "gelu":
        z = torch.empty_like(y)
        ops.native().gelu(y, z)
        y = z
    elif act == "relu":
        y = torch.relu_(y)
    elif act == "quick_gelu":
        y = y * torch.sigmoid(1.702 * y)
    return y if out_dtype in (None, y.dtype) else y.to(out_dtype)


def enable_tuned_blas() -> bool:
    import tempfile

    import torch.cuda.tunable as tunable

    path = os.path.join(ROOT, "tools", "data", "tunableop_mi355x.csv")
    tunable.enable(True)
    tunable.tuning_enable(False)
    tunable.record_untuned_enable(False)
    tunable.set_filename(os.path.join(tempfile.gettempdir(), f"gai_tunableop_{os.getpid()}.csv"))
    ok = bool(tunable.read_file(path))
    if not ok:
        tunable.enable(False)
    return ok


def patch() -> None:
    native_linear, native_rope = ops.linear, ops.linear_rope_kv

    def linear(x, w, bias=None, residual=None, act=None, out_dtype=None, out=None):
        M = x.numel() // x.shape[-1]
        if (x.is_cuda and M > 64 and residual is None and out is None and not isinstance(w, ops.Fp8Weight)
                and act not in ("geglu", "gelu_tanh")):
            y = blas_linear(x.reshape(M, x.shape[-1]), w, bias, act, out_dtype or x.dtype)
            return y.view(*x.shape[:-1], y.shape[-1])
        return native_linear(x, w, bias, residual, act, out_dtype, out)

    def linear_rope_kv(x, w, bias, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, k_scale=1.0,
                       v_scale=1.0):
        if x.numel() // x.shape[-1] <= 64:
            return native_rope(x, w, bias, positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D, k_scale,
                               v_scale)
        ops.rope_kv_write(linear(x, w, bias=bias), positions, cos_sin, slots, q_out, k_cache, v_cache, Hq, Hkv, D,
                          True, k_scale, v_scale)

    ops.linear, ops.linear_rope_kv = linear, linear_rope_kv


def main():
    argv = sys.argv[1:]
    tuned = "--tuned" in argv
    if "--" in argv:
        argv = argv[argv.index("--") + 1:]
    argv = [a for a in argv if a != "--tuned"]
    if tuned:
        print("[blas_ab] TunableOp table loaded:", enable_tuned_blas(), file=sys.stderr)
    patch()
    sys.argv = [os.path.join(ROOT, "bench.py")] + argv
    runpy.run_path(sys.argv[0], run_name="__main__")


if __name__ == "__main__":
    main()
