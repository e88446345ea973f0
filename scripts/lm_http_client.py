#!/usr/bin/env python3
"""One load-generator process for GET /inference (scripts/bench_configs.py): connects, waits for the
go file, sends ``n`` keep-alive requests back to back with seeds seed0.., prints one JSON line
(per-request latencies in ms, errors, the X-Hipzap-Path values seen). A process per client so no
client shares a GIL with another or with the server.

    python -S scripts/lm_http_client.py PORT N SEED0 GO_FILE
"""
import http.client
import json
import os
import sys
import time


def main():
    port, n, seed0, go = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
    c.connect()
    while not os.path.exists(go):
        time.sleep(0.0005)
    lat, errs, paths = [], 0, set()
    for i in range(n):
        t = time.perf_counter()
        try:
            c.request("GET", f"/inference?seed={seed0 + i}")
            r = c.getresponse()
            body = r.read()
            if r.status != 200 or not body.startswith(b'{"response": {"text": '):
                errs += 1
            paths.add(r.getheader("X-Hipzap-Path") or "wsgi")
        except (OSError, http.client.HTTPException):
            errs += 1
            c = http.client.HTTPConnection("127.0.0.1", port, timeout=120)
        lat.append((time.perf_counter() - t) * 1e3)
    print(json.dumps({"lat": lat, "errors": errs, "paths": sorted(paths), "t_end": time.time()}), flush=True)


if __name__ == "__main__":
    main()
