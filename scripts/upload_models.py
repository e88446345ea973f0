#!/usr/bin/env python3
"""Sync ./models to <models_bucket>/models (reference: scripts/upload_models.py).

Reads ``zappa_settings.json[stage].aws_environment_variables.models_bucket``; ``s3://`` buckets
use ``aws s3 sync`` when the CLI is present, local ``file://`` / directory buckets are copied."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

from hipzap.__main__ import main  # noqa: E402

if __name__ == "__main__":
    main(["upload", *sys.argv[1:]])
