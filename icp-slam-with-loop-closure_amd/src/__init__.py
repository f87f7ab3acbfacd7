"""Drop-in replacements for the reference's ``src`` modules on the hot path.

``src.icp``, ``src.pose_graph_optimization``, ``src.pose_graph`` and
``src.utils`` keep the names, signatures, return types and in-place side
effects of cohnt/ICP-SLAM-with-Loop-Closure's modules of the same name, so
``scripts/main.py`` (``import src.icp as icp`` ...) runs unchanged; the work is
done by the HIP kernels in ``slamhip``.
"""
import os as _os
import sys as _sys

_PKG_ROOT = _os.path.dirname(_os.path.dirname(_os.path.abspath(__file__)))
if _PKG_ROOT not in _sys.path:
    _sys.path.insert(0, _PKG_ROOT)
