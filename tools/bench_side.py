import json, sys
sys.path.insert(0, '.')
import bench
print(json.dumps({"kfdb": bench.kfdb_latency(), "lm": bench.local_mapping_matchers()}))
