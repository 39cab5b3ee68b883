"""The `gol` CLI reproduces the reference program's surface (Parallel_Life_MPI.cpp
main :190-240): same input files, same output.txt bytes and offsets (not
truncated, :166-170), same stdout lines (:179, :236)."""
import hashlib
import json
import os
import re
import subprocess

import pytest

from conftest import GOLDEN

GOLD = json.load(open(os.path.join(GOLDEN, "ref_outputs.json")))


def setup_dir(tmp_path, epochs, h=1500, w=500, data=None):
    if data is None:
        data = open(os.path.join(GOLDEN, "data.txt"), "rb").read()
    (tmp_path / "data.txt").write_bytes(data)
    (tmp_path / "grid_size_data.txt").write_text(f"{h} {w} {epochs}")
    return tmp_path


def run_cli(pkg, d, *args):
    return subprocess.run([pkg.CLI_PATH, "--dir", str(d), *args], capture_output=True,
                          text=True, timeout=300)


def test_zero_epochs_echo_and_no_truncate(pkg, tmp_path):
    """E = 0 needs no GPU: the reference writes the input bytes back; a longer
    pre-existing output.txt keeps its tail (no O_TRUNC)."""
    d = setup_dir(tmp_path, 0)
    stale = b"x" * (1500 * 501 + 37)
    (d / "output.txt").write_bytes(stale)
    r = run_cli(pkg, d, "--ref-ranks", "3")
    assert r.returncode == 0, r.stderr
    out = (d / "output.txt").read_bytes()
    assert out[:1500 * 501] == (d / "data.txt").read_bytes()
    assert out[1500 * 501:] == b"x" * 37
    lines = r.stdout.splitlines()
    assert lines[:3] == [f"Process {i} wrote data to the file." for i in range(3)]
    assert re.fullmatch(r"Total time = [0-9.e+-]+", lines[3])


def test_bad_config_file(pkg, tmp_path):
    (tmp_path / "grid_size_data.txt").write_text("12 x")
    r = run_cli(pkg, tmp_path)
    assert r.returncode == 1
    assert "Error reading integers from file." in r.stderr


def test_short_data_file(pkg, tmp_path):
    d = setup_dir(tmp_path, 0, data=b"0101\n")
    r = run_cli(pkg, d)
    assert r.returncode == 1


@pytest.mark.gpu
@pytest.mark.parametrize("np_,gens", [(1, 100), (4, 100), (2, 3), (8, 4)])
def test_cli_matches_reference_output(pkg, tmp_path, np_, gens):
    case = [c for c in GOLD["cases"] if c["np"] == np_ and c["gens"] == gens][0]
    d = setup_dir(tmp_path, gens)
    args = ["--ref-ranks", str(np_)] if np_ > 1 else []
    r = run_cli(pkg, d, *args)
    assert r.returncode == 0, r.stderr
    out = (d / "output.txt").read_bytes()
    assert hashlib.sha256(out).hexdigest() == case["sha256"]
    assert len(r.stdout.splitlines()) == np_ + 1


@pytest.mark.gpu
def test_cli_conway_rule(pkg, oracle, tmp_path):
    h, w = 50, 70
    g = oracle.bp_random(h, w, 2)
    data = oracle.bp_unpack(g, w)
    d = setup_dir(tmp_path, 9, h, w, data)
    r = run_cli(pkg, d, "--rule", "B3/S23")
    assert r.returncode == 0, r.stderr
    assert (d / "output.txt").read_bytes() == oracle.bp_unpack(
        oracle.bp_run(g, w, 9, oracle.CONWAY), w)


@pytest.mark.gpu
def test_cli_c2_program_surface(pkg, oracle, tmp_path):
    """(r06) C2 through the reference's program surface: a 4096 x 4096 data.txt
    (16.8 MB, the splitmix64 p = 0.5 field) and 1000 epochs in
    grid_size_data.txt; the CLI's output.txt (GPU ASCII codec in and out, the
    resident kernel between) equals the oracle's 1000 generations byte for byte."""
    n = 4096
    g = oracle.bp_random(n, n, 1)
    d = setup_dir(tmp_path, 1000, n, n, oracle.bp_unpack(g, n))
    r = run_cli(pkg, d)
    assert r.returncode == 0, r.stderr
    want = oracle.bp_unpack(oracle.bp_run(g, n, 1000, oracle.REF_RULE, threads=16), n)
    assert (d / "output.txt").read_bytes() == want
    lines = r.stdout.splitlines()
    assert lines[0] == "Process 0 wrote data to the file."
    assert re.fullmatch(r"Total time = [0-9.e+-]+", lines[1])


@pytest.mark.gpu
@pytest.mark.parametrize("stripes", [2, 5])
def test_cli_stripes_intended_semantics(pkg, tmp_path, stripes):
    """--stripes S (S row stripes with real halo exchange, one process) gives the
    reference's intended result, i.e. its -np 1 output, for any S."""
    case = [c for c in GOLD["cases"] if c["np"] == 1 and c["gens"] == 100][0]
    d = setup_dir(tmp_path, 100)
    r = run_cli(pkg, d, "--gpus", "1", "--stripes", str(stripes))
    assert r.returncode == 0, r.stderr
    assert hashlib.sha256((d / "output.txt").read_bytes()).hexdigest() == case["sha256"]


# ---- gol-mpi: the multi-process launch shape (mpirun -np P, one rank per GPU) ----

MPIRUN = "/opt/conda/bin/mpirun"


def mpi_cli(pkg):
    path = os.path.join(os.path.dirname(pkg.CLI_PATH), "gol-mpi")
    if not (os.path.exists(path) and os.path.exists(MPIRUN)):
        pytest.skip("gol-mpi not built (no MPI on this host)")
    return path


def run_mpi(pkg, d, np_, *args):
    return subprocess.run([MPIRUN, "-np", str(np_), mpi_cli(pkg), "--dir", str(d), *args],
                          capture_output=True, text=True, timeout=300)


def test_mpi_cli_usage_and_bad_config(pkg, tmp_path):
    """Argument and grid_size_data.txt errors end every rank before any GPU call."""
    r = run_mpi(pkg, tmp_path, 1, "--help")
    assert r.returncode == 0 and "gol-mpi" in r.stderr
    (tmp_path / "grid_size_data.txt").write_text("12 x")
    assert run_mpi(pkg, tmp_path, 2).returncode != 0


@pytest.mark.gpu
def test_mpi_cli_one_rank_matches_reference(pkg, tmp_path):
    """mpirun -np 1 gol-mpi: RCCL bootstrap over MPI, rank engine, its rows read and
    written at their offsets -- the reference's -np 1 output, stale tail kept.
    (Two ranks need two GPUs: RCCL refuses two ranks on one device.)"""
    case = [c for c in GOLD["cases"] if c["np"] == 1 and c["gens"] == 100][0]
    d = setup_dir(tmp_path, 100)
    (d / "output.txt").write_bytes(b"y" * (1500 * 501 + 5))
    r = run_mpi(pkg, d, 1)
    assert r.returncode == 0, r.stderr
    out = (d / "output.txt").read_bytes()
    assert hashlib.sha256(out[:1500 * 501]).hexdigest() == case["sha256"]
    assert out[1500 * 501:] == b"y" * 5
    lines = r.stdout.splitlines()
    assert lines[0] == "Process 0 wrote data to the file."
    assert re.fullmatch(r"Total time = [0-9.e+-]+", lines[1])
