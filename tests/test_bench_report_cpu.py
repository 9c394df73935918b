"""bench.py's report helpers on CPU: a kernel profiled as two sections (the DQN fc_fwd's
online and target launches) is reported as one record with each launch kept apart."""
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import bench  # noqa: E402


def _rec(name, launches, avg_us, tf, peak=833.3):
    return dict(name=name, launches=launches, avg_us=avg_us, total_ms=launches * avg_us / 1e3,
                bound="mfma", achieved=tf, unit="TFLOP/s", peak=peak, frac=round(tf / peak, 4))


def test_merge_launch_sections_sums_time_and_flops():
    online = _rec("fc_fwd", 50, 43.0, 290.0)
    target = _rec("fc_fwd_target", 50, 52.0, 120.0)
    other = _rec("conv3_fwd", 100, 29.0, 236.0)
    sections = [online, target, other]
    bench.merge_launch_sections(sections, "fc_fwd", "fc_fwd_target", ("online", "target"))
    assert [s["name"] for s in sections] == ["fc_fwd", "conv3_fwd"]
    m = sections[0]
    flops = 50 * 43.0e-6 * 290.0e12 + 50 * 52.0e-6 * 120.0e12
    secs = 50 * 43.0e-6 + 50 * 52.0e-6
    assert m["launches"] == 100
    assert abs(m["achieved"] - flops / secs / 1e12) < 0.01
    assert abs(m["avg_us"] - 47.5) < 1e-9
    assert [p["launch"] for p in m["per_launch"]] == ["online", "target"]
    assert m["per_launch"][1]["avg_us"] == 52.0


def test_merge_launch_sections_without_the_second_section_is_a_no_op():
    online = _rec("fc_fwd", 100, 43.0, 290.0)
    sections = [online]
    bench.merge_launch_sections(sections, "fc_fwd", "fc_fwd_target", ("online", "target"))
    assert sections == [online] and "per_launch" not in online
