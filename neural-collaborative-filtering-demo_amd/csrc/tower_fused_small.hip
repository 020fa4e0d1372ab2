// The fused attention block + MLP tower (tower_fused.hip) in small-batch tiles: 3 interaction
// groups (15 rows, one 16-row MFMA tile) per workgroup instead of 16 (80 rows, five tiles).
//
// Reference: the same modules (src/model/architecture.py:18-57, 230-252, 315-354) at the batch
// the reference trains with, config/config.yaml:65 (batch_size 256: 256 groups of 5 = 1,280
// rows).  In 80-row tiles that batch runs 16 workgroups on 256 CUs, each CU carrying a whole
// 80-row chain of phases (95 us for the fused backward); in 15-row tiles it
// runs 86, each with a fifth of the row work.  The device code is the same (attn_block_dev.h,
// mlp_tower_dev.h compiled with these geometry constants; internal linkage per translation unit),
// so every row's forward output is the same bits as in 80-row tiles; its input gradients agree to
// fp32 rounding (the backward's row-tile GEMMs run over another tile count) and the weight
// gradients sum the same rows in other per-workgroup groupings (fp32 rounding of the partials).
#define NCF_ATTN_G64 3
#define NCF_MLP_RT 1
#define NCF_FWD_RT 1
#define NCF_FWD_VR 16
#define NCF_TF(name) name##_small
#include "tower_fused.hip"
