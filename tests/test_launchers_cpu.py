"""The full-node launchers: every sweep validates its results, every
results directory goes through stats, and the like-for-like comparison against the reference's
published CSVs is produced. Static checks (the scripts need an 8-GPU node to run)."""

import os
import re
import subprocess

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _read(name):
    return open(os.path.join(REPO, "launch", name)).read()


def test_launchers_parse():
    for name in os.listdir(os.path.join(REPO, "launch")):
        if name.endswith(".sh"):
            subprocess.run(["bash", "-n", os.path.join(REPO, "launch", name)], check=True)


def test_collectives_sweep_validates_and_compares():
    s = _read("collectives_sweep.sh")
    sweeps = [l for l in s.splitlines() if "-m $M" in l]
    assert sweeps and all("$V" in l for l in sweeps), sweeps
    assert 'V="--validate --resume"' in s
    out_dirs = set(re.findall(r"--output-dir \$ROOT/(\S+)", s))
    stat_dirs = set(re.findall(r"--input-dir \$ROOT/(\S+)", s))
    assert out_dirs <= stat_dirs, out_dirs - stat_dirs          # MoE and direct included
    assert s.count("cli.compare") == 1 and s.count("$C --mode") == 4


def test_allreduce_variants_validate_and_compare():
    s = _read("allreduce_variants.sh")
    assert "--resume --validate" in s
    for line in s.splitlines():
        if "cli.collectives" in line:
            assert "--validate" in line or '$M' in line, line
    assert "cli.compare" in s and "cli.stats --mode 1d" in s
