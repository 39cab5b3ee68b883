"""CPU suite: the C-ABI library loads, exports every symbol include/gol.h
declares, and its host-only entry points behave (no GPU needed)."""
import ctypes
import os
import re
import subprocess

import pytest

from conftest import ROOT

HEADER = os.path.join(ROOT, "include", "gol.h")


def declared_symbols():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(gol_[a-z_]+)\s*\(", src)))


def test_header_matches_binding(pkg):
    assert declared_symbols() == sorted(pkg.EXPORTS)


def test_library_exports_every_symbol(pkg):
    L = pkg.lib()
    for name in declared_symbols():
        assert hasattr(L, name), name
    out = subprocess.run(["nm", "-D", "--defined-only", pkg.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r" T (gol_[a-z_]+)", out))
    assert set(declared_symbols()) <= exported


def test_library_is_gfx950(pkg):
    blob = open(pkg.LIB_PATH, "rb").read()
    assert b"amdgcn-amd-amdhsa--gfx950" in blob  # the embedded code object's target


def test_config_defaults(pkg):
    c = pkg.make_config()
    assert (c.birth_mask, c.survive_mask) == pkg.REF_RULE
    assert c.semantics == pkg.SEM_GLOBAL and c.device == -1 and c.tb_depth == 0


@pytest.mark.parametrize("h,n", [(65536, 8), (65536, 3), (7, 7), (10, 4), (1500, 8)])
def test_rank_rows_partition(pkg, h, n):
    rows = [pkg.rank_rows(h, n, r) for r in range(n)]
    assert rows[0][0] == 0
    for (r0, c), (r1, _) in zip(rows, rows[1:]):
        assert r0 + c == r1
    assert rows[-1][0] + rows[-1][1] == h
    assert max(c for _, c in rows) - min(c for _, c in rows) <= 1


def test_rank_rows_rejects_bad_args(pkg):
    with pytest.raises(pkg.GolError):
        pkg.rank_rows(10, 0, 0)
    with pytest.raises(pkg.GolError):
        pkg.rank_rows(10, 2, 2)


def test_bad_config_rejected_before_touching_gpu(pkg):
    for kw in ({"rule": (512, 0)}, {"tb_depth": 3}, {"handoff": 3}, {"tb_depth": 20},
               {"word_planes": 4}, {"handoff": 2, "tb_depth": 2}, {"resident": 3}):
        with pytest.raises(pkg.GolError) as ei:
            pkg.Engine(10, 10, **kw)
        assert ei.value.status == pkg.GOL_EINVAL
    with pytest.raises(pkg.GolError):
        pkg.Engine(0, 10)


def test_c_abi_from_c(pkg, tmp_path):
    """The header compiles as C and links against libgol.so (a C caller's view)."""
    src = tmp_path / "t.c"
    src.write_text(
        '#include "gol.h"\n#include <stdio.h>\n'
        "int main(void){gol_config c; gol_config_init(&c); uint64_t r0=0,n=0;\n"
        "if (gol_rank_rows(100,3,1,&r0,&n)!=GOL_OK) return 1;\n"
        "printf(\"%llu %llu %u\\n\",(unsigned long long)r0,(unsigned long long)n,c.survive_mask);"
        "return 0;}\n")
    exe = tmp_path / "t"
    subprocess.run(["gcc", "-std=c99", "-Wall", "-Werror", f"-I{ROOT}/include", str(src),
                    "-o", str(exe), f"-L{os.path.dirname(pkg.LIB_PATH)}",
                    f"-l:{os.path.basename(pkg.LIB_PATH)}",  # libgol.so, or a GOL_LIB build
                    f"-Wl,-rpath,{os.path.dirname(pkg.LIB_PATH)}"]
                   # the sanitizer build's runtime is preloaded (tools/asan_cpu_suite.sh)
                   + (["-Wl,--allow-shlib-undefined"] if os.environ.get("GOL_ASAN_SUITE") else []),
                   check=True)
    out = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout
    assert out.split() == ["34", "33", "4"]


def test_column_split_layout(tmp_path):
    """bitlayout.h: split/join are inverse permutations and gol_split_bit agrees."""
    src = tmp_path / "t.cpp"
    src.write_text(
        '#include "bitlayout.h"\n#include <cstdio>\n#include <random>\n'
        "int main(){std::mt19937_64 r(1);\n"
        " for(int i=0;i<100000;++i){uint64_t c=r(); uint64_t v=gol_split64(c);\n"
        "  if(gol_join64(v)!=c) return 1;\n"
        "  for(unsigned j=0;j<64;++j) if(((c>>j)&1)!=((v>>gol_split_bit(j))&1)) return 2;}\n"
        " if(gol_split64(1ull)!=1ull || gol_split64(2ull)!=(1ull<<32)) return 3;\n"
        " std::puts(\"ok\"); return 0;}\n")
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT}/mpi-game-of-life_amd/csrc", str(src),
                    "-o", str(exe)], check=True)
    assert subprocess.run([str(exe)], capture_output=True, text=True).stdout.strip() == "ok"


def test_four_plane_group_layout(tmp_path):
    """bitlayout.h: the 4-plane lane group (two words, 128 columns) is a bit
    permutation with column 4j+k of the group at bit j of plane k, and
    split/join are inverses; the 2-plane group is the column split."""
    src = tmp_path / "t.cpp"
    src.write_text(
        '#include "bitlayout.h"\n#include <cstdio>\n#include <random>\n'
        "int main(){std::mt19937_64 r(2);\n"
        " for(int i=0;i<100000;++i){uint64_t c[2]={r(),r()},s[2],b[2];\n"
        "  gol_split_group(c,s,4); gol_join_group(s,b,4);\n"
        "  if(b[0]!=c[0]||b[1]!=c[1]) return 1;\n"
        "  for(unsigned col=0;col<128;++col){unsigned k=col&3,j=col>>2;\n"
        "   uint64_t plane=(s[k>>1]>>(32*(k&1)))&0xFFFFFFFFull;\n"
        "   if(((c[col>>6]>>(col&63))&1)!=((plane>>j)&1)) return 2;}\n"
        "  gol_split_group(c,s,2); if(s[0]!=gol_split64(c[0])) return 3;\n"
        "  gol_join_group(s,b,2); if(b[0]!=c[0]) return 4;}\n"
        " std::puts(\"ok\"); return 0;}\n")
    exe = tmp_path / "t"
    subprocess.run(["g++", "-O2", "-std=c++17", f"-I{ROOT}/mpi-game-of-life_amd/csrc", str(src),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    assert r.stdout.strip() == "ok", r.returncode


def test_shipped_library_has_only_product_kernels(pkg):
    """The default build instantiates 2-plane stencil kernels of depths 1..16 only
    (auto_layout's depths and the remainder launches); the 4-plane lane groups and
    depths 20/24/32 live in the dev build (make dev)."""
    blob = open(pkg.LIB_PATH, "rb").read()
    names = set(re.findall(rb"life_tb_kernelILi(\d+)ELi(\d)ELi(\d)ELb(\d)E", blob))
    depths = {int(k) for k, _, _, _ in names}
    assert depths == {1, 2, 4, 6, 7, 8, 12, 16}
    assert {int(n) for _, _, n, _ in names} == {2}
    assert {(int(k), int(h)) for k, _, _, h in names if int(h)} == {(k, 1) for k in (4, 6, 7, 8, 12, 16)}
    # (r06) no multi-pass instantiation (template flag MP = true): dev build only
    full = set(re.findall(rb"life_tb_kernelILi(\d+)ELi(\d)ELi(\d)ELb(\d)ELi(\d)ELb(\d)E", blob))
    assert full and {mp for *_, mp in full} == {b"0"}
    # the resident kernel: 5 rows-per-wavefront variants x 3 rule kinds
    res = set(re.findall(rb"life_res_kernelILi(\d)ELi(\d)E", blob))
    assert res == {(str(m).encode(), str(r).encode()) for m in (2, 3, 4, 6, 8) for r in range(3)}
