for i in 1 2 3; do
 for L in liborbx_base.so liborbx.so; do
  ORBX_LIB=orb_slam_2_ros_amd/$L timeout -k 10 200 python bench.py --no-extras --no-profile 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read().strip().splitlines()[-1]); print('$L', d['value'])" || exit 1
 done
done
