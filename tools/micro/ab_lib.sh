# A/B of two builds of libigx.so on the C4 ablation: the in-tree library vs $1 (a variant .so)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python tools/ablate_c4.py > gpurun_out/ab_base.log 2>&1 || { echo base failed; tail gpurun_out/ab_base.log; exit 1; }
cp inspektor-gadget_amd/libigx.so /tmp/libigx_base.so
cp "$1" inspektor-gadget_amd/libigx.so
timeout -k 10 300 python tools/ablate_c4.py > gpurun_out/ab_var.log 2>&1 || { echo var failed; tail gpurun_out/ab_var.log; exit 1; }
cp /tmp/libigx_base.so inspektor-gadget_amd/libigx.so
echo "base: $(tail -1 gpurun_out/ab_base.log)"
echo "var:  $(tail -1 gpurun_out/ab_var.log)"
