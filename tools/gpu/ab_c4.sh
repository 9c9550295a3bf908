# C4 per-pass A/B: per-kernel times of config c4 under several settings
#   bash tools/gpu/ab_c4.sh "tag:ENV=V,ENV=V" ...   (IGX_LIB=<path> selects another build)
set -o pipefail
export KT_ROWS=${KT_ROWS:-8}
for spec in "$@"; do
  tag=${spec%%:*}; envs=${spec#*:}
  bash tools/gpu/ktrace.sh "$tag" c4 IGX_X=0 ${envs//,/ } || exit 1
done
