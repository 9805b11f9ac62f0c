"""po_brax_amd -- MI355X-native rollout engine for po-brax's partially observable Ant tasks.

Import surface mirrors ``po_brax``: ``po_brax_amd.envs`` (create / create_fn /
create_gym_env / the three env classes / wrappers), ``po_brax_amd.standard_observability_masks``
and ``po_brax_amd.jumpy`` (device threefry RNG).  All compute runs in libpob.so (HIP, gfx950).
"""
__version__ = "0.1.0"
