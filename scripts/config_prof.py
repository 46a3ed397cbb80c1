"""Time named BASELINE configs of bench.py alone (for rocprofv3 runs):
python scripts/config_prof.py c2_10k_F8 [more names]; prints config_rates' JSON."""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


class Args:
    seed = 1
    max_heartbeats = 400
    msg_size = 15000
    config_traffic_json = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles",
                                       "config_traffic_latest.json")


bench.CONFIGS = {k: v for k, v in bench.CONFIGS.items() if k in sys.argv[1:]}
print(json.dumps(bench.config_rates(Args, 0)))
