"""Generate one Markdown page per public class/function of rocket_amd from its docstrings.

    python docs/create_api_md.py            # writes docs/api/*.md and docs/api/index.md

(The reference generates Sphinx autoclass stubs from ``rocket.core.__sphinx_classes__``; here the
pages are plain Markdown so they render without a docs toolchain.)
"""

from __future__ import annotations

import inspect
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

SECTIONS = {
    "Capsules (rocket_amd.core)": ["rocket_amd.core"],
    "Runtime": ["rocket_amd.runtime.engine", "rocket_amd.runtime.graphs", "rocket_amd.runtime.data",
                "rocket_amd.runtime.host_data", "rocket_amd.runtime.comm", "rocket_amd.runtime.profiling",
                "rocket_amd.runtime.trackers", "rocket_amd.runtime.checkpoint_io"],
    "Parallel": ["rocket_amd.parallel.ddp", "rocket_amd.parallel.flat_grads", "rocket_amd.parallel.rccl"],
    "Ops (HIP kernels)": ["rocket_amd.ops.cross_entropy", "rocket_amd.ops.optim", "rocket_amd.ops.lenet",
                          "rocket_amd.ops.norm", "rocket_amd.ops.activation", "rocket_amd.ops.linear",
                          "rocket_amd.ops.conv", "rocket_amd.ops.data"],
    "Models": ["rocket_amd.models.lenet", "rocket_amd.models.resnet", "rocket_amd.models.vit"],
}


def _public(mod):
    names = getattr(mod, "__all__", None) or [n for n in dir(mod) if not n.startswith("_")]
    out = []
    for n in names:
        obj = getattr(mod, n, None)
        if (inspect.isclass(obj) or inspect.isfunction(obj)) and getattr(obj, "__module__", "").startswith(
                mod.__name__.rsplit(".", 1)[0] if mod.__name__.endswith("core") else mod.__name__):
            out.append((n, obj))
    return out


def _page(name, obj) -> str:
    lines = [f"# `{obj.__module__}.{name}`", ""]
    try:
        lines += [f"```python\n{name}{inspect.signature(obj)}\n```", ""]
    except (TypeError, ValueError):
        pass
    lines += [inspect.getdoc(obj) or "(no docstring)", ""]
    if inspect.isclass(obj):
        for mname, m in inspect.getmembers(obj, inspect.isfunction):
            if mname.startswith("_") or m.__qualname__.split(".")[0] != obj.__name__:
                continue
            doc = inspect.getdoc(m)
            try:
                sig = str(inspect.signature(m))
            except (TypeError, ValueError):
                sig = "(...)"
            lines += [f"## `{mname}{sig}`", "", doc or "", ""]
    return "\n".join(lines)


def main() -> None:
    import importlib

    out_dir = os.path.join(ROOT, "docs", "api")
    os.makedirs(out_dir, exist_ok=True)
    index = ["# API reference", ""]
    for section, mods in SECTIONS.items():
        index += [f"## {section}", ""]
        for mname in mods:
            mod = importlib.import_module(mname)
            for name, obj in _public(mod):
                fn = f"{mod.__name__}.{name}.md"
                with open(os.path.join(out_dir, fn), "w") as fh:
                    fh.write(_page(name, obj))
                index.append(f"* [`{mod.__name__}.{name}`]({fn})")
        index.append("")
    with open(os.path.join(out_dir, "index.md"), "w") as fh:
        fh.write("\n".join(index))
    print(f"wrote {len(os.listdir(out_dir))} pages to {out_dir}")


if __name__ == "__main__":
    main()
