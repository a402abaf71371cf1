"""TensorBoard launcher (reference start_tensorboard at
mnist_keras_distributed.py:192-197: in-process server on $TB_PORT, default 6006).

If the ``tensorboard`` package is importable it is launched in-process on
TB_PORT.  Otherwise a minimal stdlib HTTP server serves the scalar summaries of
``logdir`` (read with the native TFRecord/Event reader) as JSON at
``/data/scalars`` and a tiny HTML table at ``/`` — enough to watch loss /
accuracy / global_step/sec while training.
"""
from __future__ import annotations

import json
import logging
import os
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer
from pathlib import Path

log = logging.getLogger("tensorflow_distributed_example_amd")


def _collect(logdir):
    from ..io.events import read_events
    runs = {}
    for f in sorted(Path(logdir).rglob("events.out.tfevents.*")):
        run = str(f.parent.relative_to(logdir)) or "."
        try:
            evs = read_events(f)
        except Exception:
            continue
        for e in evs:
            for tag, v in e.get("scalars", {}).items():
                runs.setdefault(run, {}).setdefault(tag, []).append([e.get("wall_time", 0), e.get("step", 0), v])
    return runs


class _Handler(BaseHTTPRequestHandler):
    logdir = "."

    def log_message(self, *a):
        pass

    def do_GET(self):
        data = _collect(self.logdir)
        if self.path.startswith("/data/scalars"):
            body = json.dumps(data).encode()
            ctype = "application/json"
        else:
            rows = []
            for run, tags in data.items():
                for tag, pts in tags.items():
                    last = pts[-1]
                    rows.append(f"<tr><td>{run}</td><td>{tag}</td><td>{last[1]}</td><td>{last[2]:.6g}</td></tr>")
            body = ("<html><body><h3>tde scalars: %s</h3><table border=1><tr><th>run</th><th>tag</th><th>step</th>"
                    "<th>value</th></tr>%s</table></body></html>" % (self.logdir, "".join(rows))).encode()
            ctype = "text/html"
        self.send_response(200)
        self.send_header("Content-Type", ctype)
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)


class ScalarServer:
    def __init__(self, logdir, port):
        handler = type("H", (_Handler,), {"logdir": str(logdir)})
        self.httpd = ThreadingHTTPServer(("0.0.0.0", port), handler)
        self.port = self.httpd.server_address[1]
        self.thread = threading.Thread(target=self.httpd.serve_forever, daemon=True, name="tde-tensorboard")

    def launch(self):
        self.thread.start()
        return f"http://localhost:{self.port}/"

    def shutdown(self):
        self.httpd.shutdown()


def start_tensorboard(logdir, port=None):
    """Start a TensorBoard (or the built-in scalar viewer) on TB_PORT in a background thread."""
    port = int(os.getenv("TB_PORT", 6006)) if port is None else port
    try:
        from tensorboard import program as tb_program  # noqa: F401
        tb = tb_program.TensorBoard()
        tb.configure(logdir=str(logdir), port=port)
        url = tb.launch()
        log.info("Starting TensorBoard with --logdir=%s", logdir)
        return url
    except Exception:
        srv = ScalarServer(logdir, port)
        url = srv.launch()
        log.info("Starting TensorBoard (built-in scalar viewer) with --logdir=%s at %s", logdir, url)
        return srv
