# Build the current csrc (or a copy in SRCDIR) into a side library
# (tools/ab/NAME.so) without touching the in-tree libg2k_hip.so: the A/B arm
# of tools/bench_lib.py.
#   [SCENE_FLAGS="..."] tools/build_lib_variant.sh NAME [SRCDIR]   (extra flags for g2k_scene.hip)
set -e
SRC=${2:-multimodaltraj_2_amd/csrc}
O=tools/ab/build_$1; mkdir -p $O
for f in $SRC/*.hip; do
  b=$(basename $f .hip); x=""; [ $b = g2k_scene ] && x="-mllvm -disable-lsr $SCENE_FLAGS"
  /opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -fno-slp-vectorize -std=c++17 -fPIC -Iinclude $x -c -o $O/$b.o $f &
done
g++ -O2 -std=c++17 -fPIC -Wall -Iinclude -c -o $O/g2k_walk.o $SRC/g2k_walk.cpp
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o tools/ab/$1.so $O/*.o
rm -rf $O
echo tools/ab/$1.so
