// SnapshotV1 emission on the device (emit.hip): parameters and launcher.
#pragma once
#include <hip/hip_runtime.h>

#include "engine_types.hpp"

namespace mte {
struct EmitParams {
    // the documents of this launch (doc indices) and the replay's final state (Engine::finish)
    const u32* list;
    u32 n_list;
    u32 chunk;                 // SnapshotV1 chunk size in characters (10000)
    u32 legacy;                // 1: SnapshotLegacy header / body chunks (snapshotlegacy.ts) instead of SnapshotV1
    const DocRes* res;
    const DocCfg* cfg;
    const uint4* vis;          // rows: (len, seq, removedSeq, client | removedClient << 8 | flags)
    const uint4* aux;          // rows: (map, text offset in the doc's run | marker refType, ...)
    const u32* maps;           // the property map of every row with props (map_words per row), or null
    u32 map_words;
    const u16* text;           // gathered text of every row
    u32* esc;                  // per row: its text's JSON byte size + flags (engine_types.hpp ESC_*):
                               // written by COUNT, read by WRITE
    // property text tables (interned JSON texts of keys and values)
    const char* key_text;
    const u64* key_off;
    const unsigned char* key_is_index;
    const u32* key_index;
    const char* val_text;
    const u64* val_off;
    const u32* val_flags;
    const u32* val_objidx;
    const u64* val_objmatch;
    // client names by slot, JSON-quoted UTF-8: document d's slots are name_off[name_base[d] ..]
    const char* names;
    const u64* name_off;
    const u64* name_base;
    // scratch
    uint4* ent;                // legacy: snapshot entries, indexed like the rows; SnapshotV1: the chunk
                               // table (per chunk: first entry, entry count, length in characters)
    u16* tscr;                 // gathered text of runs that span elided rows, indexed like `text`
    // per document (indexed by doc): COUNT writes, WRITE reads
    u32* n_ent;
    u64* size;
    u32* nblobs;
    // WRITE
    char* out;
    const u64* out_off;
    u64* blob_off;
    const u64* blob_base;
};
hipError_t launch_emit(const EmitParams& p, bool write, hipStream_t s);
}  // namespace mte
