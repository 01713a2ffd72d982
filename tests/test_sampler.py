"""The Python statistical profiler (ncc/sampler.py): off without NCC_PY_SAMPLE; with it, SIGPROF samples of
the running stacks are counted and written as JSON at exit."""
import json
import os
import signal

from ncc import sampler


def test_sampler_is_off_without_the_variable(monkeypatch):
    monkeypatch.delenv("NCC_PY_SAMPLE", raising=False)
    assert sampler.start("x") is False


def test_sampler_counts_stacks_and_dumps_json(tmp_path, monkeypatch):
    dumps = []
    monkeypatch.setattr(sampler.atexit, "register", dumps.append)
    monkeypatch.setenv("NCC_PY_SAMPLE", str(tmp_path / "py"))
    monkeypatch.setenv("NCC_PY_SAMPLE_US", "100")
    monkeypatch.setattr(sampler, "_n", [0])
    monkeypatch.setattr(sampler, "_self", sampler.Counter())
    monkeypatch.setattr(sampler, "_incl", sampler.Counter())
    monkeypatch.setattr(sampler, "_stacks", sampler.Counter())
    old = signal.getsignal(signal.SIGPROF)
    try:
        assert sampler.start("unit")

        def busy_loop():
            x = 0
            for i in range(3_000_000):
                x += i % 7
            return x
        while sampler._n[0] < 5:
            busy_loop()
        assert len(dumps) == 1
        dumps[0]()  # the atexit hook: stops the timer and writes the file
    finally:
        signal.setitimer(signal.ITIMER_PROF, 0, 0)
        signal.signal(signal.SIGPROF, old)
    out = tmp_path / f"py.unit.{os.getpid()}.json"
    data = json.loads(out.read_text())
    assert data["samples"] >= 5 and data["interval_us"] == 100
    assert any("busy_loop" in k for k in data["self"]) and any("busy_loop" in k for k in data["inclusive"])
    assert any(s.endswith("busy_loop") for s in data["stacks"])
    sampler._on_prof(signal.SIGPROF, None)  # a signal without a frame is ignored
