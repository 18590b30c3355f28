/* Force-included (-include) into the prebuilt binaries the GPU box cannot
 * rebuild: keeps "SMG_SOURCE_HASH=<hash of the sources>" in the binary
 * (math_amd/srchash.py checks it against the tree at run time). */
#ifndef SMG_SOURCE_TAG_H
#define SMG_SOURCE_TAG_H
#ifdef SMG_SOURCE_HASH
__attribute__((used)) static const char smg_source_tag_[] = "SMG_SOURCE_HASH=" SMG_SOURCE_HASH;
#endif
#endif
