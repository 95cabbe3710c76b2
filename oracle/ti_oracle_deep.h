/*
 * ti_oracle_deep.h -- TEST INFRASTRUCTURE ONLY.  The oracle decode step at full depth
 * (ti_oracle_deep.c): or_decode_step's arithmetic on group-quantized weights held as int8 +
 * fp16 group scales instead of materialised fp32, multi-threaded along independent outputs.
 */
#ifndef TI_ORACLE_DEEP_H
#define TI_ORACLE_DEEP_H

#include "ti_oracle.h"

#ifdef __cplusplus
extern "C" {
#endif

typedef struct or_qmodel or_qmodel;

/* or_model_synth's model (bits 4 or 8, group scales); NULL for other bit widths */
or_qmodel* or_qmodel_synth(const or_model_config* cfg, uint64_t seed, float norm_jitter);
void or_qmodel_free(or_qmodel* m);
/* or_model_fill_kv */
void or_qmodel_fill_kv(or_qmodel* m, int n, uint64_t seed);
int or_qmodel_len(const or_qmodel* m);
int or_qmodel_set_len(or_qmodel* m, int n);
/* or_decode_step(kv_round_f16 = 1): logits [vocab], returns the argmax (-1 past max_seq) */
int or_qmodel_step(or_qmodel* m, int token, float* logits);

#ifdef __cplusplus
}
#endif
#endif
