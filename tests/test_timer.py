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
