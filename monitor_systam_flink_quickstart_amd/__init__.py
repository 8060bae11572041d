"""Import alias: ``monitor_systam_flink_quickstart_amd`` is the ``mxstream`` package.

``import monitor_systam_flink_quickstart_amd.api`` etc. resolve to the same module objects as
``mxstream.api`` (models/ ops/ parallel/ utils/ runtime/ api/ oracle/)."""
import importlib
import sys

import mxstream as _mx

__version__ = _mx.__version__
for _sub in ("api", "models", "ops", "parallel", "runtime", "utils", "oracle"):
    _mod = importlib.import_module(f"mxstream.{_sub}")
    sys.modules[f"{__name__}.{_sub}"] = _mod
    globals()[_sub] = _mod
