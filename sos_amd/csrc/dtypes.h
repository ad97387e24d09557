// dtypes.h -- the SOS datatype/op contract as seen by the HIP kernels.
//
// SOS dispatches the local combine on (datatype, op) in shmem_internal_reduce_local
// (src/shmem_internal_op.h:305-339).  Datatypes fall into three op classes
// (src/shmem_internal_op.h:225-303):
//   FP   : char, signed char, ptrdiff_t, float, double, long double -> min max sum prod
//   CPLX : float _Complex, double _Complex                          -> sum prod
//   INT  : every other integer type                                 -> all seven ops
// SIGNED_BYTE and FORTRAN_INTEGER reach the default case ("invalid data type").
//
// On the device every type reduces to a storage class: its width, whether a compare
// is signed, and whether it is floating point.  Sum/prod/bitwise results of integer
// types depend only on the width (two's-complement wrap), so they share unsigned
// kernels; only min/max need the signedness.
#pragma once
#include <stddef.h>
#include "sosx.h"

enum SosKind {
    K_INVALID = 0,
    K_S8, K_U8, K_S16, K_U16, K_S32, K_U32, K_S64, K_U64,
    K_F32, K_F64, K_C32, K_C64, K_LDBL
};

enum SosClass { C_NONE = 0, C_FP, C_CPLX, C_INT };

struct SosDtypeInfo {
    int kind;
    int cls;
    size_t size;
};

// Indexed by shm_internal_datatype_t (src/transport.h:19-49), LP64 x86-64 sizes.
static inline SosDtypeInfo sos_dtype_info(int dt)
{
    static const SosDtypeInfo tab[SOSX_DT_COUNT] = {
        /* SIGNED_BYTE     */ {K_INVALID, C_NONE, 0},
        /* CHAR (signed)   */ {K_S8, C_FP, 1},
        /* SCHAR           */ {K_S8, C_FP, 1},
        /* SHORT           */ {K_S16, C_INT, 2},
        /* INT             */ {K_S32, C_INT, 4},
        /* LONG            */ {K_S64, C_INT, 8},
        /* LONG_LONG       */ {K_S64, C_INT, 8},
        /* FORTRAN_INTEGER */ {K_INVALID, C_NONE, 0},
        /* INT8            */ {K_S8, C_INT, 1},
        /* INT16           */ {K_S16, C_INT, 2},
        /* INT32           */ {K_S32, C_INT, 4},
        /* INT64           */ {K_S64, C_INT, 8},
        /* PTRDIFF_T       */ {K_S64, C_FP, 8},
        /* UCHAR           */ {K_U8, C_INT, 1},
        /* USHORT          */ {K_U16, C_INT, 2},
        /* UINT            */ {K_U32, C_INT, 4},
        /* ULONG           */ {K_U64, C_INT, 8},
        /* ULONG_LONG      */ {K_U64, C_INT, 8},
        /* UINT8           */ {K_U8, C_INT, 1},
        /* UINT16          */ {K_U16, C_INT, 2},
        /* UINT32          */ {K_U32, C_INT, 4},
        /* UINT64          */ {K_U64, C_INT, 8},
        /* SIZE_T          */ {K_U64, C_INT, 8},
        /* FLOAT           */ {K_F32, C_FP, 4},
        /* DOUBLE          */ {K_F64, C_FP, 8},
        /* LONG_DOUBLE     */ {K_LDBL, C_FP, 16},
        /* FLOAT_COMPLEX   */ {K_C32, C_CPLX, 8},
        /* DOUBLE_COMPLEX  */ {K_C64, C_CPLX, 16},
    };
    if (dt < 0 || dt >= SOSX_DT_COUNT) return SosDtypeInfo{K_INVALID, C_NONE, 0};
    return tab[dt];
}

static inline int sos_check_op(int op, int dt)
{
    SosDtypeInfo d = sos_dtype_info(dt);
    if (d.kind == K_INVALID) return SOSX_ERR_DTYPE;
    switch (d.cls) {
        case C_FP:
            return (op == SOSX_OP_MIN || op == SOSX_OP_MAX || op == SOSX_OP_SUM ||
                    op == SOSX_OP_PROD) ? SOSX_OK : SOSX_ERR_OP;
        case C_CPLX:
            return (op == SOSX_OP_SUM || op == SOSX_OP_PROD) ? SOSX_OK : SOSX_ERR_OP;
        case C_INT:
            return (op >= SOSX_OP_BAND && op <= SOSX_OP_PROD) ? SOSX_OK : SOSX_ERR_OP;
        default:
            return SOSX_ERR_DTYPE;
    }
}
