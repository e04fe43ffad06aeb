"""The pure-JS CPU baseline (oracle/lz4_js.mjs, our restatement of the reference's
block codec, timed by bench.py) is bit-exact on the reference's golden vectors:
every golden raw block compresses to the reference's bytes and decodes back, and
the 4 MiB digest rows match. CPU only (node)."""
import json
import os
import shutil
import subprocess

import pytest

import oracle as O
from conftest import GOLDEN, ROOT, cases_of

NODE = shutil.which("node")
pytestmark = pytest.mark.skipif(NODE is None, reason="node is not installed")


def test_js_restatement_matches_golden_blocks(manifest, tmp_path):
    rows = []
    for c in cases_of(manifest, "block"):
        if "gen" in c:
            g = c["gen"]
            src = O.generate(g["gen"], g["seed"], g["n"])
        else:
            with open(os.path.join(GOLDEN, c["src_file"]), "rb") as f:
                src = f.read()
        p = tmp_path / (c["name"] + ".bin")
        p.write_bytes(bytes(src))
        rows.append({"name": c["name"], "src": str(p), "comp_len": c["comp_len"], "comp_xxh": c["comp_xxh"]})
    job = tmp_path / "job.json"
    job.write_text(json.dumps(rows))
    lib = os.path.join(ROOT, "oracle", "lz4_js.mjs")
    script = f"""
import fs from 'fs';
import {{ compressBlock, decompressBlock }} from '{lib}';
const rows = JSON.parse(fs.readFileSync('{job}', 'utf8'));
const out = [];
for (const r of rows) {{
  const src = new Uint8Array(fs.readFileSync(r.src));
  const dst = new Uint8Array(src.length + (src.length / 255 | 0) + 16);
  const n = compressBlock(src, dst, 0, src.length, new Int32Array(16384), 0);
  const back = new Uint8Array(src.length);
  const w = decompressBlock(dst, 0, n, back, 0);
  out.push({{ name: r.name, n, comp: Buffer.from(dst.subarray(0, n)).toString('base64'),
             rt: w === src.length && Buffer.from(back).equals(Buffer.from(src)) }});
}}
console.log(JSON.stringify(out));
"""
    r = subprocess.run([NODE, "--no-warnings", "--input-type=module", "-e", script], capture_output=True, text=True,
                       timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    import base64
    import numpy as np
    got = json.loads(r.stdout.strip().splitlines()[-1])
    for want, g in zip(rows, got):
        comp = np.frombuffer(base64.b64decode(g["comp"]), dtype=np.uint8)
        assert g["n"] == want["comp_len"], g["name"]
        assert "%08x" % O.xxh32(comp) == want["comp_xxh"], g["name"]
        assert g["rt"], g["name"]


def test_js_baseline_harness_checks_reference_digests():
    """The timing harness itself verifies its compressor on the reference's 4 MiB digests."""
    r = subprocess.run([NODE, "--no-warnings", os.path.join(ROOT, "oracle", "js_cpu_baseline.mjs"), "tiles216", "2", "2",
                        os.path.join(GOLDEN, "manifest.json")], capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-3000:]
    d = json.loads(r.stdout.strip().splitlines()[-1])
    assert d["verified"] and d["golden_digests_checked"] == 4 and d["threads"] == 2
