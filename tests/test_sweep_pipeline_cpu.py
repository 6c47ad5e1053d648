"""1D / 3D sweep -> stats -> compare end to end on the CPU (gloo, world 2): the same pipeline
the ranks-on-one-GPU and multi-GPU tests run (tests/sweep_pipeline.py)."""

from sweep_pipeline import check_pipeline, run_pipeline


def test_collectives_sweep_pipeline_gloo_cpu(tmp_path):
    res = run_pipeline(tmp_path, 2, backend="gloo", device="cpu", timeout=600)
    check_pipeline(res, 2)
