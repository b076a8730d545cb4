// Test-infrastructure driver for the reference's CPUTests/BVHConstructTest
// (compiled unmodified, -Dmain=bvhct_ref_main: its `void main` becomes an
// ordinary function).  Runs it (Karras 2012 Fig. 3 keys, main.cpp:259-265) and
// dumps the reference's node array: bvhct_nodes.i32 = 15 x {parent, childL, childR, code}.
#include <cstdio>
#include <cstdlib>

struct ref_node { int parent; int childL, childR; unsigned code; };
extern ref_node nodes[];
void bvhct_ref_main();

int main(int argc, char** argv) {
    const char* dir = argc > 1 ? argv[1] : ".";
    bvhct_ref_main();
    char path[4096];
    snprintf(path, sizeof(path), "%s/bvhct_nodes.i32", dir);
    FILE* f = fopen(path, "wb");
    if (!f) { perror(path); return 1; }
    fwrite(nodes, sizeof(ref_node), 15, f);
    fclose(f);
    return 0;
}
