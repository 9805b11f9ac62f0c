"""``brax.io.html`` for engine envs: a standalone page embedding the trajectory JSON and
brax's three.js viewer (the page the reference's notebooks display, ant_tag.ipynb:449)."""
from __future__ import annotations

from typing import Sequence

from . import json as _bjson

_VIEWER = "https://cdn.jsdelivr.net/gh/google/brax@v0.0.10/js/viewer.js"

_TEMPLATE = """<html>
  <head>
    <title>brax visualizer</title>
    <style>
      body {{
        margin: 0;
        padding: 0;
      }}
      #brax-viewer {{
        margin: 0;
        padding: 0;
        height: {height}px;
      }}
    </style>
  </head>
  <body>
    <script type="application/javascript">
    var system = {system};
    </script>
    <div id="brax-viewer"></div>
    <script type="module">
      import {{Viewer}} from '{viewer}';
      const domElement = document.getElementById('brax-viewer');
      var viewer = new Viewer(domElement, system);
    </script>
  </body>
</html>
"""


def render(env, qps: Sequence, height: int = 480, env_index: int = 0) -> str:
    """HTML page for one env's trajectory (``brax.io.html.render(sys, qps, height)``)."""
    return _TEMPLATE.format(height=int(height), system=_bjson.dumps(env, qps, env_index), viewer=_VIEWER)


def save_html(path: str, env, qps: Sequence, make_dir: bool = False, env_index: int = 0) -> None:
    import os
    if make_dir:
        os.makedirs(os.path.dirname(os.path.abspath(path)), exist_ok=True)
    with open(path, "w") as f:
        f.write(render(env, qps, env_index=env_index))
