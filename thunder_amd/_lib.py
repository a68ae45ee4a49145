"""ctypes binding of libthunder_amd.so (the C-ABI declared in include/thunder_amd.h).

There is no fallback: if the HIP library is missing or fails to load, every
entry point raises.  Build it with ``python -m thunder_amd.build`` (or
``__graft_entry__.build()``).
"""
import ctypes
import os

from .build import LIB

_c_int, _c_float, _c_double, _c_size = ctypes.c_int, ctypes.c_float, ctypes.c_double, ctypes.c_size_t
_p = ctypes.c_void_p

# name -> (restype, argtypes); mirrors include/thunder_amd.h
SIGNATURES = {
    "thx_abi_version": (_c_int, []),
    "thx_last_error": (ctypes.c_char_p, []),
    "thx_pixel_set": (_c_int, [_c_int, _c_int, _c_float, _c_float, _c_int, _p, _p, _p, _p, _p]),
    "thx_ctf": (_c_int, [_p, _c_int, _p, _p, _c_int, _c_int, _p, _p]),
    "thx_trans_table": (_c_int, [_p, _c_int, _p, _p, _c_int, _c_int, _p, _p]),
    "thx_rotmat": (_c_int, [_p, _c_int, _p, _p]),
    "thx_project3d": (_c_int, [_p, _c_int, _c_int, _p, _c_int, _p, _p, _c_int, _p, _p]),
    "thx_dvp": (_c_int, [_p, _c_int, _p, _c_int, _p, _p, _p, _c_int, _c_int, _p, _p]),
    "thx_global_scan_workspace": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "thx_global_scan": (_c_int, [_p, _c_int, _p, _c_int, _p, _p, _p, _c_int, _c_int, _p, _p,
                                 _c_int, _c_int, _p, _p, _p, _p, _c_int, _p, _c_size, _p]),
    "thx_global_scan_dvp": (_c_int, [_p, _c_int, _p, _c_int, _p, _p, _p, _c_int, _c_int, _p, _p,
                                     _c_int, _c_int, _p, _p, _p, _p, _c_int, ctypes.c_float, _p, _p,
                                     _c_size, _p]),
    "thx_local_phase_workspace": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "thx_view_order_workspace": (_c_size, [_c_int]),
    "thx_view_order": (_c_int, [_c_int, _c_int, _p, _p, _p, _c_size, _p]),
    "thx_volume_cells": (_c_int, [_p, _c_int, _p, _p]),
    "thx_pixel_tile_order": (_c_int, [_p, _p, _c_int, _c_int, _p, _p]),
    "thx_local_phase": (_c_int, [_p, _c_int, _c_int, _c_int, _p, _c_int, _p, _c_int, _p, _p, _p, _p, _p,
                                 _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p, _p, _p, _p,
                                 _c_size, _p]),
    "thx_defocus_pre": (_c_int, [_p, _c_int, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p]),
    "thx_ctf_search": (_c_int, [_p, _p, _p, _c_int, _p, _p, _p, _c_int, _c_int, _p, _p]),
    "thx_local_phase_d": (_c_int, [_p, _p, _c_int, _c_int, _c_int, _p, _c_int, _p, _c_int, _c_int,
                                   _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int,
                                   _c_int, _p, _p, _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_pf_defocus": (_c_int, [_c_int, _c_int, _c_int, _c_double, ctypes.c_ulonglong, ctypes.c_uint,
                                _p, _p, _p, _p]),
    "thx_expectation_ctf_workspace": (_c_size, [_p, _p, _c_int, _c_int, _c_int]),
    "thx_expectation_ctf": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _p, _p,
                                     _p, _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_global_sample_sizes": (_c_int, [_c_int, _c_int, _c_int, _c_double, _c_double, _p, _p, _p]),
    "thx_global_sample_set": (_c_int, [_c_int, _c_int, _c_double, ctypes.c_ulonglong, _p, _p, _p, _p,
                                       _p]),
    "thx_resample": (_c_int, [_c_int, _c_int, _p, _p, _c_int, _p, _p, _p, _p, _p]),
    "thx_pf_resample_workspace": (_c_size, [_c_int, _c_int]),
    "thx_pf_resample": (_c_int, [_c_int, _c_int, _c_int, _p, _c_int, _p, _c_int, ctypes.c_ulonglong,
                                 ctypes.c_uint, _c_int, _p, _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_pf_calvari": (_c_int, [_c_int, _c_int, _p, _c_int, _p, _c_double, _c_double, _p, _p, _p]),
    "thx_pf_balance_rot": (_c_int, [_c_int, _c_int, _p, _p, _p]),
    "thx_global_sample_set2d": (_c_int, [_c_int, _c_int, _c_double, ctypes.c_ulonglong, _p, _p, _p,
                                         _p, _p]),
    "thx_volume_ypair": (_c_int, [_p, _c_int, _p, _p]),
    "thx_fft3d_workspace": (_c_size, [_c_int]),
    "thx_fft3d": (_c_int, [_p, _p, _c_int, _c_int, _c_int, _p, _c_size, _p]),
    "thx_pf_acg_mean": (_c_int, [_c_int, _c_int, _p, _c_int, _p, _p, _p]),
    "thx_pf_calvari2d": (_c_int, [_c_int, _c_int, _p, _c_int, _p, _c_double, _c_double, _p, _p, _p]),
    "thx_pf_balance_rot2d": (_c_int, [_c_int, _c_int, _p, _p, _p]),
    "thx_pf_perturb2d": (_c_int, [_c_int, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _c_double,
                                  _c_double, _c_double, ctypes.c_ulonglong, ctypes.c_uint, _p]),
    "thx_expectation2d_workspace": (_c_size, [_p, _c_int, _c_int]),
    "thx_expectation2d_ctf_workspace": (_c_size, [_p, _p, _c_int, _c_int]),
    "thx_expectation2d_ctf": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p,
                                       _p, _p, _p, _c_size, _p]),
    "thx_local_phase2d_d_workspace": (_c_size, [_c_int, _c_int, _c_int, _c_int]),
    "thx_local_phase2d_d": (_c_int, [_p, _c_int, _c_int, _p, _p, _c_int, _p, _c_int, _c_int, _p, _p,
                                     _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _p, _p, _p,
                                     _p, _p, _p, _p, _c_size, _p]),
    "thx_expectation2d": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _p, _p,
                                   _p, _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_pf_peak": (_c_int, [_c_int, _c_int, _p, _c_int, _p, _c_int, _p]),
    "thx_insert3d": (_c_int, [_p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _p, _c_int,
                              _c_int, _p, _p, _c_int, _c_int, _p]),
    "thx_insert3d_workspace": (_c_size, [_c_int, _c_int, _c_int]),
    "thx_insert3d_tiled": (_c_int, [_p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _p, _c_int,
                                    _c_int, _p, _p, _p, _c_int, _c_int, _c_int, _p, _c_size, _p]),
    "thx_insert3d_binned_workspace": (_c_size, [_c_int, _c_int, _c_int, _c_int, _c_int]),
    "thx_insert3d_binned": (_c_int, [_p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _p,
                                     _c_int, _c_int, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _p,
                                     _c_size, _p]),
    "thx_insert3d_binned_d": (_c_int, [_p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _p,
                                       _p, _c_int, _c_int, _p, _p, _p, _c_int, _c_int, _c_int,
                                       _c_int, _p, _c_size, _p]),
    "thx_InsertFTCS": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_float,
                                _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p]),
    "thx_rccl_unique_id": (_c_int, [_p]),
    "thx_rccl_comm_init": (_c_int, [_c_int, _p, _c_int, _p]),
    "thx_rccl_comm_destroy": (_c_int, [_p]),
    "thx_halfmap_allreduce": (_c_int, [_p, _p, _p, _p, _p, ctypes.c_longlong, _c_int, _p]),
    "thx_halfmap_sendrecv": (_c_int, [_p, _p, ctypes.c_longlong, _c_int, _p, ctypes.c_longlong,
                                      _c_int, _p]),
    "thx_project2d": (_c_int, [_p, _c_int, _c_int, _p, _c_int, _p, _p, _c_int, _p, _p]),
    "thx_local_phase2d_workspace": (_c_size, [_c_int, _c_int, _c_int]),
    "thx_local_phase2d": (_c_int, [_p, _c_int, _c_int, _p, _p, _c_int, _p, _c_int, _p, _p, _p, _p, _p,
                                   _p, _p, _p, _c_int, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _c_size,
                                   _p]),
    "thx_insert2d": (_c_int, [_p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _p, _c_int,
                              _c_int, _p, _p, _c_int, _c_int, _p]),
    "thx_ExpectGlobal2D": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int,
                                    _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int]),
    "thx_InsertI2D": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p,
                               _c_float, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int,
                               _c_int]),
    "thx_insert2d_d": (_c_int, [_p, _p, _p, _p, _c_int, _c_int, _p, _p, _p, _p, _p, _p, _p, _p,
                                _c_int, _c_int, _p, _p, _c_int, _c_int, _p]),
    "thx_adapter_devices": (_c_int, [_p, _c_int, _p]),
    "thx_adapter_device_policy": (_c_int, [_c_int, _c_int, ctypes.c_char_p, _c_int, _c_int, _p, _c_int, _p]),
    "thx_set_device": (_c_int, [_c_int]),
    "thx_img_stats": (_c_int, [_p, _c_int, _c_int, _c_int, _c_float, _p, _p, _p]),
    "thx_img_finish": (_c_int, [_p, _c_int, _c_int, _c_float, _c_float, _c_int, _c_float,
                                ctypes.c_ulonglong, _p, _p, _p, _p]),
    "thx_remask": (_c_int, [_p, _c_int, _c_int, _c_float, _c_float, _p, _p]),
    "thx_img_gather": (_c_int, [_p, _c_int, _c_int, _p, _c_int, _p, _p]),
    "thx_ctf_image": (_c_int, [_p, _c_int, _c_int, _p, _p]),
    "thx_reconstruct_workspace": (_c_size, [_c_int, _c_int]),
    "thx_reconstruct": (_c_int, [_p, _p, _c_int, _c_int, _c_float, _c_float, _c_int, _c_int, _c_int, _p,
                                 _c_int, _c_int, _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_symmetry": (_c_int, [ctypes.c_char_p, _c_int, _p, _p, _p]),
    "thx_symmetrize_ft": (_c_int, [_p, _p, _c_int, _c_int, _p, _c_int, ctypes.c_double, _p]),
    "thx_prepare_tf_workspace": (_c_size, [_c_int]),
    "thx_prepare_tf": (_c_int, [_p, _p, _c_int, _p, _c_int, _c_int, _c_int, _p, _c_size, _p]),
    "thx_pf_symmetrise": (_c_int, [_c_int, _c_int, _p, _c_int, _p, _p, _c_int, ctypes.c_ulonglong,
                                   ctypes.c_uint, _p]),
    "thx_prepare_tf2d": (_c_int, [_p, _p, _c_int, _c_int, _p]),
    "thx_reconstruct2d_workspace": (_c_size, [_c_int, _c_int, _c_int]),
    "thx_reconstruct2d": (_c_int, [_p, _p, _c_int, _c_int, _c_int, _c_float, _c_float, _c_int, _c_int,
                                   _p, _c_int, _c_int, _p, _p, _p, _c_size, _p]),
    "thx_fsc_workspace": (_c_size, [_c_int]),
    "thx_fsc": (_c_int, [_p, _p, _c_int, _c_int, _p, _p, _c_size, _p]),
    "thx_expectation_workspace": (_c_size, [_p, _c_int, _c_int, _c_int]),
    "thx_expectation": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int,
                                 _p, _p, _p, _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_local_phase_routed": (_c_int, [_p, _p, _p, _c_int, _c_int, _p, _c_int, _p, _c_int, _p, _p, _p,
                                        _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _p, _p,
                                        _p, _p, _p, _p, _p, _c_size, _p]),
    "thx_local_phase_sel": (_c_int, [_p, _p, _c_int, _c_int, _c_int, _p, _c_int, _p, _c_int, _p, _p, _p,
                                     _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _p, _p, _p,
                                     _p, _p, _p, _c_size, _p]),
    "thx_event_pairs_create": (_c_int, [_c_int, _p]),
    "thx_event_pairs_elapsed": (_c_int, [_p, _c_int, _p]),
    "thx_event_pairs_destroy": (_c_int, [_p, _c_int]),
    "thx_getAviDevice": (_c_int, [_p, _c_int, _p]),
    "thx_ExpectPreidx": (_c_int, [_c_int, _p, _p, _p, _p, _c_int]),
    "thx_ExpectPrefre": (_c_int, [_c_int, _p, _p, _c_int]),
    "thx_ExpectLocalIn": (_c_int, [_c_int, _p, _p, _p, _p, _c_int, _c_int, _c_int]),
    "thx_tex_create": (_c_int, [_c_int, _c_int, _c_int, _p]),
    "thx_tex_destroy": (_c_int, [_p]),
    "thx_ExpectLocalV3D": (_c_int, [_c_int, _p, _p, _c_int]),
    "thx_ExpectLocalV2D": (_c_int, [_c_int, _p, _p, _c_int]),
    "thx_ExpectLocalPreI2D": (_c_int, [_c_int, _c_int, _p, _p, _p, _p, _p, _p, _c_float, _c_float,
                                       _c_float, _c_float, _c_int, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExpectLocalP": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int,
                                  _c_int]),
    "thx_ExpectLocalHostA": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int,
                                      _c_int, _c_int]),
    "thx_calpoint_create": (_c_int, [_c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _c_int, _p]),
    "thx_calpoint_destroy": (_c_int, [_p]),
    "thx_ExpectLocalRTD": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _p]),
    "thx_ExpectLocalPreI3D": (_c_int, [_c_int, _c_int, _p, _p, _p, _p, _p, _p, _c_float, _c_float,
                                       _c_float, _c_float, _c_int, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExpectLocalM": (_c_int, [_c_int, _c_int, _p, _p, _p, _p, _p, _p, _p, _p, _c_double,
                                  _c_int]),
    "thx_ExpectLocalHostF": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int]),
    "thx_ExpectLocalFin": (_c_int, [_c_int, _p, _p, _p, _p, _p, _c_int]),
    "thx_ExpectFreeIdx": (_c_int, [_c_int, _p, _p]),
    "thx_ExpectRotran": (_c_int, [_p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExpectProject": (_c_int, [_p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExpectGlobal3D": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int,
                                    _c_int, _c_int, _c_int, _c_int]),
    "thx_InsertFT": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int,
                              _c_int, _c_int, _c_int, _c_int]),
    "thx_InsertFTC": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int,
                               _c_int, _c_int, _c_int, _c_int]),
    "thx_InsertFTComm": (_c_int, [_p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int,
                                  _c_int, _c_int, _c_int, _c_int, _p]),
    # reconstruction host adapters (Interface.h:320-528)
    "thx_PrepareTF": (_c_int, [_c_int, _p, _p, _p, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExposePT": (_c_int, [_c_int, _p, _c_int, _c_int, _c_int, _p, _c_int, _c_int, _c_int]),
    "thx_ExposePT2D": (_c_int, [_c_int, _p, _c_int, _c_int, _c_int, _p, _c_int, _c_int, _c_int]),
    "thx_ExposeWT": (_c_int, [_c_int, _p, _p, _p, _c_float, _c_int, _c_float, _c_int, _c_int, _c_int,
                              _c_int, _c_int, _c_int, _p]),
    "thx_ExposeWT2D": (_c_int, [_c_int, _p, _p, _p, _c_float, _c_int, _c_float, _c_int, _c_int, _c_int,
                                _c_int, _c_int, _c_int, _p]),
    "thx_ExposeWT_T": (_c_int, [_c_int, _p, _p, _c_int, _c_int, _c_int]),
    "thx_ExposeWT2D_T": (_c_int, [_c_int, _p, _p, _c_int, _c_int, _c_int]),
    "thx_AllocDevicePoint": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int]),
    "thx_HostDeviceInit": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int,
                                    _c_int]),
    "thx_ExposeC": (_c_int, [_c_int, _p, _p, _p, _p, _p, _c_int, _c_int]),
    "thx_ExposeForConvC": (_c_int, [_c_int, _p, _p, _p, _p, _c_float, _c_int, _c_float, _c_int, _c_int,
                                    _c_int, _c_int]),
    "thx_ExposeWC": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _c_int, _c_int, _c_int, _c_int]),
    "thx_FreeDevHostPoint": (_c_int, [_c_int, _p, _p, _p, _p, _p, _p, _p, _p, _p, _c_int, _c_int]),
    "thx_ExposePFW": (_c_int, [_c_int, _p, _p, _p, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExposePF": (_c_int, [_c_int, _p, _p, _p, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExposePF2D": (_c_int, [_c_int, _p, _p, _p, _c_int, _c_int, _c_int, _c_int]),
    "thx_ExposeCorrF": (_c_int, [_c_int, _p, _p, _c_float, _c_int]),
    "thx_ExposeCorrFT": (_c_int, [_c_int, _p, _p, _p, _c_float, _c_int]),
    "thx_ExposeCorrF2D": (_c_int, [_c_int, _p, _p, _p, _c_float, _c_int]),
    "thx_TranslateI": (_c_int, [_c_int, _p, _c_double, _c_double, _c_double, _c_int, _c_int]),
    "thx_TranslateI2D": (_c_int, [_c_int, _p, _c_double, _c_double, _c_int, _c_int]),
    "thx_ReMask": (_c_int, [_p, _c_float, _c_float, _c_float, _c_int, _c_int]),
    "thx_GCTFinit": (_c_int, [_p, _p, _c_float, _c_int, _c_int]),
}

_lib = None


class ThxError(RuntimeError):
    pass


def lib():
    """Load libthunder_amd.so (raises if it is absent: no CPU fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    path = os.environ.get("THX_LIB", LIB)   # override: A/B builds in tools/microbench.py
    if not os.path.exists(path):
        raise ThxError(f"{path} is missing: run `python -m thunder_amd.build` "
                       "(the HIP path has no fallback)")
    L = ctypes.CDLL(path)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(L, name)
        fn.restype = res
        fn.argtypes = args
    _lib = L
    return L


def check(status, what=""):
    if status != 0:
        msg = lib().thx_last_error().decode(errors="replace")
        raise ThxError(f"{what} failed (status {status}): {msg}")
