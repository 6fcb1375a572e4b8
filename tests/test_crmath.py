"""pcp_crmath.h -- the device's correctly rounded atan2 (a faithful first result, then the
midpoint tests in double-double) -- against the running glibc, whose atan2 the reference and the
oracle call.  CPU only.  glibc 2.35 rounds atan2 correctly except near ties (its slow paths are
gone): the checker's mismatches are those ties, ~4e-4 of the pairs, where the x87 long-double
atan2l sides with the correctly rounded value (tools/libm_cr_check.py)."""
import shutil
import subprocess
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


@pytest.fixture(scope="module")
def checker(tmp_path_factory):
    cc = shutil.which("gcc") or shutil.which("cc")
    if cc is None:
        pytest.skip("no C compiler")
    exe = tmp_path_factory.mktemp("crmath") / "crmath_check"
    subprocess.run([cc, "-O2", "-ffp-contract=off", f"-I{ROOT / 'pointcloud_processor_amd' / 'csrc'}",
                    str(ROOT / "tests" / "libm" / "crmath_check.c"), "-o", str(exe), "-lm"],
                   check=True)
    return exe


def test_cr_atan2_acos_sin_match_glibc_but_near_ties(checker):
    """4 M pairs, first results one ulp off either way or exact: the fix returns glibc's value
    for all but glibc's near-tie misroundings (< 1e-3 of the pairs)."""
    r = subprocess.run([str(checker), "4000000"], capture_output=True, text=True, timeout=300,
                       check=True)
    lines = {l.split()[0]: list(map(int, l.split()[1:])) for l in r.stdout.splitlines()}
    n, bad, skipped = lines["atan2"]
    assert n > 3_800_000 and bad < 1e-3 * n, r.stdout
    # acos (0, 1) and sin [2^-20, pi / 2] (not yet used by a kernel): glibc's misroundings near
    # ties are ~1e-3 of the arguments (the x87 acosl / sinl side with the correctly rounded value
    # in ~5 of 6 of the disagreements; the rest lie within the x87's own error)
    for fn in ("acos", "sin"):
        n, bad, _ = lines[fn]
        assert n == 4_000_000 and bad < 3e-3 * n, r.stdout
    # the scoring's composite sin(M_PI / 2 - acos(d)) (pcp_score_sin_part, round 6): glibc's value
    # but for its near ties; the fast phase never decides against the exact path (20 M
    # arguments: 0 of 20,000,000), and hands fewer than 1e-3 of the arguments to it
    n, bad, disagree, slow = lines["spa"]
    assert n == 4_000_000 and bad < 3e-3 * n and disagree == 0 and slow < 1e-3 * n, r.stdout
