"""clore-tx against the reference's own util test vectors (test/util/data/clore-util-test.json,
read in place from the reference checkout: every case's arguments, stdin, expected hex / JSON output
and exit code). The vectors carry Bitcoin-style addresses and keys, so they run with the 0 / 5 / 128
version bytes they were generated with."""
import io
import json
import os

import pytest

from nodexa_chain_core_amd.cli import clore_tx

DATA = "/root/reference/test/util/data"
PREFIXES = ["-pubkeyprefix=0", "-scriptprefix=5", "-secretprefix=128"]


def _cases():
    path = os.path.join(DATA, "clore-util-test.json")
    if not os.path.exists(path):
        return []
    return [c for c in json.load(open(path)) if c.get("exec", "").endswith("clore-tx")]


@pytest.mark.skipif(not _cases(), reason="reference util vectors not present")
@pytest.mark.parametrize("case", _cases(), ids=lambda c: " ".join(c["args"])[:60])
def test_util_vector(case, capsys):
    args = list(case["args"])
    flags = [a for a in args if a.startswith("-") and a != "-"]
    rest = [a for a in args if not (a.startswith("-") and a != "-")]
    stdin = io.StringIO(open(os.path.join(DATA, case["input"])).read()) if "input" in case else None
    out = io.StringIO()
    rc = clore_tx.main(PREFIXES + flags + rest, stdin=stdin, stdout=out)
    assert rc == case.get("return_code", 0), capsys.readouterr().err
    if "output_cmp" in case:
        want = open(os.path.join(DATA, case["output_cmp"])).read()
        if case["output_cmp"].endswith(".json"):
            assert json.loads(out.getvalue()) == json.loads(want)
        else:
            assert out.getvalue().strip() == want.strip()
