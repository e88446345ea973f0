#!/bin/bash
# Bootstrap (reference: install_all.sh): build the gfx950 native library in-tree, create the
# settings file from the template and the local models directory.
set -euo pipefail
cd "$(dirname "$0")"
python -m pip install -r requirements.txt --no-deps 2>/dev/null || echo "(offline: using preinstalled packages)"
python -m hipzap.build
[ -f zappa_settings.json ] || cp zappa_settings.rename.json zappa_settings.json
mkdir -p models
python -m hipzap info
