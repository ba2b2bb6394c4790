"""Record the reference's plugin interface signatures as data (development container only):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_plugin_signatures.py [/root/reference]

Imports ``BaseUnifiedRenderer`` and ``SharedNeRFModel`` from the reference's
``src/benchmark/base_renderer.py`` (90-281, 16-87) and writes, for every public
method and for ``__init__``, its parameter names, kinds and defaults, whether it
is abstract, and the class attributes ``__init__`` sets, to
``plugin_signatures.json``.  tests/test_host_logic.py checks the MI355X plugin
against it.  Only the interface description is committed, no source.
"""
import inspect
import json
import os
import sys
import types


def main(ref="/root/reference"):
    sys.path.insert(0, ref)
    import src  # noqa: F401

    bp = types.ModuleType("src.benchmark")
    bp.__path__ = [os.path.join(ref, "src", "benchmark")]
    sys.modules["src.benchmark"] = bp
    from src.benchmark.base_renderer import BaseUnifiedRenderer, SharedNeRFModel

    out = {}
    for cls in (BaseUnifiedRenderer, SharedNeRFModel):
        meths = {}
        for name, fn in inspect.getmembers(cls, predicate=inspect.isfunction):
            if name.startswith("_") and name != "__init__":
                continue
            sig = inspect.signature(fn)
            meths[name] = {
                "params": [{"name": p.name, "kind": str(p.kind),
                            "default": None if p.default is inspect.Parameter.empty else repr(p.default)}
                           for p in sig.parameters.values()],
                "abstract": bool(getattr(fn, "__isabstractmethod__", False)),
            }
        out[cls.__name__] = meths
    # attributes the constructor sets (a throwaway concrete subclass)
    class _Probe(BaseUnifiedRenderer):
        def execute_volume_rendering(self, *a):
            pass

        def render_image(self, *a):
            pass

    probe = _Probe("probe", "cpu")
    out["BaseUnifiedRenderer.__init__.attributes"] = sorted(k for k in vars(probe))
    out["BaseUnifiedRenderer.__init__.values"] = {k: repr(getattr(probe, k)) for k in ("near", "far", "device")}
    path = os.path.join(os.path.dirname(os.path.abspath(__file__)), "plugin_signatures.json")
    with open(path, "w") as f:
        json.dump(out, f, indent=1, sort_keys=True)
    print("wrote", path)


if __name__ == "__main__":
    main(*sys.argv[1:2])
