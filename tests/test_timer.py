"""Timer-section C ABI without a GPU (gls_timer_*): the enable switch
round-trips, a reset empties the tally, the report has its header."""
import glsamd


def test_timer_abi_cpu():
    was = glsamd.timer_enable(True)
    try:
        assert glsamd.timer_enable(True) is True
        glsamd.timer_reset()
        assert glsamd.timer_sections() == {}
        rep = glsamd.timer_report()
        assert rep.split()[:5] == ["section", "calls", "host", "ms", "GPU"]
        assert glsamd.timer_enable(False) is True
        assert glsamd.timer_enable(False) is False
    finally:
        glsamd.timer_enable(was)


def test_timer_scope_cpu():
    """A caller-opened section (MyScope: gls_timer_begin / _end) is tallied
    under its name, nested sections separately."""
    was = glsamd.timer_enable(True)
    try:
        glsamd.timer_reset()
        with glsamd.timer_scope("newton::solve"):
            with glsamd.timer_scope("direct::solve"):
                pass
        with glsamd.timer_scope("newton::solve"):
            pass
        t = glsamd.timer_sections()
        assert t["newton::solve"]["calls"] == 2 and t["direct::solve"]["calls"] == 1
        assert t["newton::solve"]["host_ms"] >= t["direct::solve"]["host_ms"] >= 0
        assert "newton::solve" in glsamd.timer_report()
    finally:
        glsamd.timer_enable(was)
        glsamd.timer_reset()
