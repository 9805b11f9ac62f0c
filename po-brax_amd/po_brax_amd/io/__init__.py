"""Trajectory export in brax's visualiser formats (``brax.io.json`` / ``brax.io.html``).

``config.brax_config(env)`` rebuilds the brax ``Config`` of an engine env as the JSON dict
the reference's notebooks embed (``notebooks/ant_tag.ipynb:449``); ``json.dumps`` /
``html.render`` / ``html.save_html`` wrap it with per-frame body poses of one env.
"""
from . import config, html, json  # noqa: F401
