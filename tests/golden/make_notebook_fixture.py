"""Extract the golden trajectory embedded in the reference notebook into a fixture.

Test infrastructure only.  Run here (where /root/reference exists):

    python tests/golden/make_notebook_fixture.py

Source: ``notebooks/ant_tag.ipynb:449`` (cell 3 output; an identical copy sits at
``notebooks/ant_heavenhell.ipynb:423``).  The cell that produced it is
``notebooks/ant_tag.ipynb:470-477``: ``rng = prngkey(0)``, an un-jitted (numpy-path,
float64) ``AntTagEnv.reset``, then 20 jitted steps.  The output is the brax
visualiser payload ``{"config": <brax.Config as JSON>, "pos": [21][12][3],
"rot": [21][12][4]}``.  We keep it verbatim as data (config + per-frame body poses),
which is what the reference's own artefact holds -- no reference source is copied.
"""
import json
import os
import sys

SRC = "/root/reference/notebooks/ant_tag.ipynb"
DST = os.path.join(os.path.dirname(os.path.abspath(__file__)), "ant_tag_notebook_trajectory.json")


def main() -> int:
    nb = json.load(open(SRC))
    html = "".join(nb["cells"][3]["outputs"][0]["data"]["text/html"])
    start = html.find('{"config"')
    obj, _ = json.JSONDecoder().raw_decode(html[start:])
    out = {
        "source": "notebooks/ant_tag.ipynb:449 (cell 3 output, brax html.render payload)",
        "config": obj["config"],
        "pos": obj["pos"],
        "rot": obj["rot"],
    }
    with open(DST, "w") as f:
        json.dump(out, f, separators=(",", ":"))
    print("wrote", DST, os.path.getsize(DST), "bytes")
    return 0


if __name__ == "__main__":
    sys.exit(main())
