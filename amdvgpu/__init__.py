"""Import alias for the ``4paradigm-k8s-device-plugin_amd`` package.

The package directory carries the project name required by the repository layout,
which is not a valid Python identifier. This shim re-points the ``amdvgpu`` package
path at that directory so every module is imported exactly once, under
``amdvgpu.<sub>``.
"""
import os as _os

_PKG_DIR = _os.path.join(_os.path.dirname(_os.path.dirname(_os.path.abspath(__file__))),
                         "4paradigm-k8s-device-plugin_amd")
__path__ = [_PKG_DIR]  # noqa: F821 - package path redirect
with open(_os.path.join(_PKG_DIR, "__init__.py")) as _f:
    exec(compile(_f.read(), _os.path.join(_PKG_DIR, "__init__.py"), "exec"))
