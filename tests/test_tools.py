"""CPU checks of the GPU measurement tooling (tools/recipes.py, tools/ab.py): the recipes the
round's evidence was made with are listed and parse their arguments (no GPU step runs)."""
import subprocess
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent


def test_recipes_list():
    p = subprocess.run([sys.executable, "tools/recipes.py", "--list"], cwd=ROOT, capture_output=True,
                       text=True, timeout=60)
    assert p.returncode == 0, p.stderr
    names = [ln.split()[0] for ln in p.stdout.splitlines() if ln.strip()]
    assert names == sorted(["ab", "check", "configs", "counters", "parts", "refresh", "shardprobe", "sizes"])


def test_recipe_ab_passes_its_options_to_ab_py(monkeypatch, tmp_path):
    sys.path.insert(0, str(ROOT / "tools"))
    import recipes
    calls = []
    monkeypatch.setattr(recipes, "run", lambda cmd, limit, *a, **k: calls.append((cmd, limit)))
    ns = recipes.argparse.Namespace(lib=["a=libplk.so"], venv=["q=PLK_TAIL_QUAD=0"], args=["--log-n 12"],
                                    tests=[], env=["PLK_LIB_ANY_SRC=1"], reps=3, limit=500)
    recipes.r_ab(tmp_path, ns)
    (cmd, limit), = calls
    assert limit == 500 and cmd[1:4] == ["-u", "tools/ab.py", "--out"]
    for flag, val in (("--lib", "a=libplk.so"), ("--venv", "q=PLK_TAIL_QUAD=0"),
                      ("--args", "--log-n 12"), ("--env", "PLK_LIB_ANY_SRC=1"), ("--reps", "3")):
        assert cmd[cmd.index(flag) + 1] == val


def test_rx_asm_gen_header_is_current(tmp_path, monkeypatch):
    """dusk-plonk_amd/csrc/rx_asm_gen.hpp is what tools/gen_rx_asm.py writes (the asm-column
    operand lists must cover every column shape ffr.hpp's rx_col_order produces)."""
    sys.path.insert(0, str(ROOT / "tools"))
    try:
        import gen_rx_asm
    finally:
        sys.path.pop(0)
    out = tmp_path / "rx_asm_gen.hpp"
    monkeypatch.setattr(gen_rx_asm, "OUT", out)
    gen_rx_asm.main()
    assert out.read_text() == (ROOT / "dusk-plonk_amd" / "csrc" / "rx_asm_gen.hpp").read_text()
