#!/bin/bash
# Recreate _refbase/ (git-ignored): the read-only reference package plus stand-ins for its two
# dependencies that are not installed here (adict, termcolor), for bench/reference_baseline.py.
set -e
cd "$(dirname "$0")/.."
rm -rf _refbase && mkdir -p _refbase/shims/adict _refbase/shims/termcolor
cp -r /root/reference/rocket _refbase/rocket
cat > _refbase/shims/adict/__init__.py <<'PY'
class adict(dict):
    """attribute-access dict (stand-in for the `adict` package)"""
    def __getattr__(self, k):
        try:
            return self[k]
        except KeyError:
            return None
    def __setattr__(self, k, v):
        self[k] = v
    def __delattr__(self, k):
        self.pop(k, None)
PY
cat > _refbase/shims/termcolor/__init__.py <<'PY'
def colored(text, *args, **kwargs):
    return text
PY
echo "refbase ok"
