set -e
mkdir -p gpurun_out
O=gpurun_out/diag1.txt
: > $O
T="timeout -k 10 120 python tools/tail_diag.py"
$T mono 640 480 1000 1024 >> $O 2>&1
for s in 1 2 3; do echo "DBG_STOP=$s" >> $O; ORBX_DBG_STOP=$s $T mono 640 480 1000 1024 >> $O 2>&1; done
echo "MATCH_CLOCKS" >> $O
ORBX_MATCH_CLOCKS=1 $T mono 640 480 1000 1024 3 2>&1 | tail -4 >> $O
for p in 32 64 128; do $T stereo 1920 1080 1000 $p >> $O 2>&1; done
cat $O
