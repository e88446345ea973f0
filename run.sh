#!/bin/bash
# Local dev server on 0.0.0.0:8082 (reference: run.sh -> python3.6 main.py)
cd "$(dirname "$0")"
export FLASK_APP=main.py
exec python main.py
