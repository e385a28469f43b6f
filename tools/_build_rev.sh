# Build the library of a git revision as an experiment variant: tools/_build_rev.sh REV NAME
# -> coeb-slam_amd/lib/var_NAME.so (A/B baselines for tools/_kab.sh; loaded with COEB_LIB_PATH).
set -eu
cd "$(dirname "$0")/.."
rev=$1; name=$2
tmp=$(mktemp -d)
git archive "$rev" coeb-slam_amd/csrc include data | tar -x -C "$tmp"
make -s -C "$tmp/coeb-slam_amd/csrc" -j8 LIB="$PWD/coeb-slam_amd/lib/var_$name.so"
rm -rf "$tmp"
echo "built lib/var_$name.so from $(git rev-parse --short "$rev")"
