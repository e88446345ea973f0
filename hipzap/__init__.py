"""hipzap — an MI355X-native (gfx950 / CDNA4) serverless-style PyTorch inference runtime.

Capabilities of gdoteof/pytorch-zappa-serverless (Flask/Zappa WSGI app that cold-loads a
state_dict and serves predictions), rebuilt around hand-written HIP kernels, hipGraph warm
paths and RCCL data parallelism. See README.md and SURVEY.md.
"""
__version__ = "0.1.0"
