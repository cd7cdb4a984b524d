/*
 * lmi_h5.h — C-ABI of liblmi_h5.so: the HDF5 files around the LMI search hot
 * path, native, over the image's libhdf5 (no h5py).
 *
 * Replaces, in the reference:
 *   - the dataset / query loaders  np.array(h5py.File(path, "r")[key])
 *     (search/search.py:48-49 for kind/key, :79-87 for clip768v2 'emb');
 *   - the result writer store_results (search/li/utils.py:85-97), whose file
 *     eval/eval.py reads: attrs algo, data, buildtime, querytime, size, params
 *     (strings as h5py writes Python str: variable-length UTF-8 scalars;
 *     floats as f64 scalars) and datasets knns (uint32 [nq][k]) and dists
 *     (float64 [nq][k]).
 * Host memory only; return 0 or an LMI_E_* code (lmi_h5_last_error() gives text).
 */
#ifndef LMI_H5_H
#define LMI_H5_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define LMI_H5_F32 0
#define LMI_H5_F16 1
#define LMI_H5_F64 2
#define LMI_H5_U32 3
#define LMI_H5_I64 4
#define LMI_H5_OTHER 9

/* Shape of dataset `name` in `path`: rank 1 or 2 (dims_out[1] = 1 for rank 1)
 * and its stored element type (LMI_H5_*). */
int lmi_h5_dataset_info(const char* path, const char* name, int64_t* dims_out,
                        int32_t* dtype_out);

/* Rows [row0, row0 + nrows) of a rank-2 floating dataset, converted by HDF5
 * to float32 (clip768v2 'emb' is stored as float16), into out[nrows][cols]. */
int lmi_h5_read_f32(const char* path, const char* name, int64_t row0, int64_t nrows,
                    float* out);

/* The same rows in the STORED floating type, as np.array(h5py.File(path)[name])
 * returns them (search.py:48-49, :79-87: clip768v2 'emb' stays float16, which
 * decides the reference's float64 arithmetic, utils.py:11): elem_bytes must be
 * the stored element size (2, 4 or 8, from lmi_h5_dataset_info); the bytes
 * are copied unconverted (little-endian IEEE, or little-endian integers: a
 * result file's uint32 knns). */
int lmi_h5_read_stored(const char* path, const char* name, int64_t row0, int64_t nrows,
                       int32_t elem_bytes, void* out);

/* store_results (utils.py:85-97): creates/truncates `path` (the parent
 * directory must exist). */
int lmi_h5_write_results(const char* path, const uint32_t* knns, const double* dists,
                         int64_t nq, int32_t k, const char* algo, const char* data,
                         double buildtime, double querytime, const char* size,
                         const char* params);

/* A rank-2 dataset `name` [rows][cols] of host float32 `buf`, stored as
 * float16 (dtype LMI_H5_F16, the SISAP'23 clip768v2 'emb' layout) or float32
 * (LMI_H5_F32, e.g. 'pca96'); the file is created, or opened for append when
 * `append` is nonzero.  Used to lay synthetic data out as the reference's
 * data/<kind>/<size>/{dataset,query}.h5 files. */
int lmi_h5_write_f32(const char* path, const char* name, int32_t dtype, int64_t rows,
                     int64_t cols, const float* buf, int32_t append);

/* The same with the caller's bytes stored unconverted: elem_bytes 2 (IEEE
 * binary16, e.g. a float16 'emb' array), 4 or 8 (little-endian IEEE).  HDF5's
 * software float32 -> float16 conversion of lmi_h5_write_f32 is slow at
 * 10M x 768; this writes at file speed. */
int lmi_h5_write_stored(const char* path, const char* name, int32_t elem_bytes, int64_t rows,
                        int64_t cols, const void* buf, int32_t append);

const char* lmi_h5_last_error(void);

#ifdef __cplusplus
}
#endif
#endif
