# Build libmapsum_base.so from the committed (HEAD) kernel sources next to the working-tree
# libmapsum.so, for same-box A/B runs (tools/ab.sh).  Run from the repo root.
set -e
C=map-reduced-approach-for-vietnamese-long-document-summarization_amd/csrc
T=$(mktemp -d)
git archive HEAD $C include | tar -x -C $T
make -C $T/$C -j8 OUT=$PWD/map-reduced-approach-for-vietnamese-long-document-summarization_amd/mapsum/libmapsum_base.so > /dev/null
rm -rf $T
