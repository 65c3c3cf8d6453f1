! ocn_sw_c.f90 -- ISO_C_BINDING interface to libocn_sw (include/ocn_sw.h).
!
! This is the "thin C-ABI shim" a Fortran PSyKAl host binds instead of the nvfortran
! gpu/kernel path: each kernel entry keeps the reference kernel's argument order
! (kernel/shallow_water/*.f90) with the 8 bounds folded into type(ocn_block) and arrays
! passed as device addresses (type(c_ptr), value).
module ocn_sw_c
    use iso_c_binding
    implicit none
    public

    integer(c_int), parameter :: OCN_OK = 0

    ! field ids (include/ocn_sw.h)
    integer(c_int), parameter :: OCN_LU = 0, OCN_LUU = 1, OCN_LUH = 2, OCN_LCU = 3, OCN_LCV = 4, OCN_LLU = 5,  &
                                 OCN_LLV = 6, OCN_DX = 7, OCN_DY = 8, OCN_DXT = 9, OCN_DYT = 10, OCN_DXH = 11, &
                                 OCN_DYH = 12, OCN_DXB = 13, OCN_DYB = 14, OCN_RLH_S = 15, OCN_R_DISS = 16,   &
                                 OCN_NUM_R4 = 17
    integer(c_int), parameter :: OCN_SSH = 32, OCN_SSHN = 33, OCN_SSHP = 34, OCN_UBRTR = 35, OCN_UBRTRN = 36,  &
                                 OCN_UBRTRP = 37, OCN_VBRTR = 38, OCN_VBRTRN = 39, OCN_VBRTRP = 40,             &
                                 OCN_HHQ = 41, OCN_HHQ_P = 42, OCN_HHQ_N = 43, OCN_HHU = 44, OCN_HHU_P = 45,    &
                                 OCN_HHU_N = 46, OCN_HHV = 47, OCN_HHV_P = 48, OCN_HHV_N = 49, OCN_HHH = 50,    &
                                 OCN_HHH_P = 51, OCN_HHH_N = 52, OCN_HHQ_REST = 53, OCN_VORT = 54,              &
                                 OCN_STR_T = 55, OCN_STR_S = 56, OCN_MU = 57, OCN_RHSX = 58, OCN_RHSY = 59,     &
                                 OCN_RHSX_ADV = 60, OCN_RHSY_ADV = 61, OCN_RHSX_DIF = 62, OCN_RHSY_DIF = 63,    &
                                 OCN_FIELD_END = 64
    ! tracer storage (core/ocean.f90:38-41): flux_x, flux_y, then ff1/ff1p/ff1n of tracer k at
    ! OCN_TRACER_BASE + 3*(k-1) + 0/1/2
    integer(c_int), parameter :: OCN_FLUX_X = 64, OCN_FLUX_Y = 65, OCN_TRACER_BASE = 66
    integer(c_int), parameter :: OCN_STAGE_CHECK_SSH_ERR = 10
    integer(c_int), parameter :: OCN_TSTAGE_TRAN_DIFF_FLUXES = 0, OCN_TSTAGE_TRAN_DIFF_TRACER = 1, &
                                 OCN_TSTAGE_TRACER_NEXT_STEP = 2
    ! execution options (ocn_ctx_set_option / ocn_ctx_get_option)
    integer(c_int32_t), parameter :: OCN_OPT_GRAPH = 1, OCN_OPT_OVERLAP = 2, OCN_OPT_STAGE_TIMING = 3,        &
                                     OCN_OPT_FUSED = 4, OCN_OPT_COMPACT = 5, OCN_OPT_MARCH = 6, OCN_OPT_FLIP = 7,  &
                                     OCN_OPT_RECOMPUTE = 8, OCN_OPT_ONEPASS = 9, OCN_OPT_KNOWN_CONSTANTS = 10,     &
                                     OCN_OPT_ONEPASS_LAST = 11, OCN_OPT_LAZY_TAIL = 12, OCN_OPT_X2 = 13,           &
                                     OCN_OPT_BATCH = 14, OCN_OPT_PAIR = 15, OCN_OPT_MULTI = 16,                    &
                                     OCN_OPT_TRACER_STEP = 17, OCN_OPT_MULTI_SPIN = 18, &
                                     OCN_OPT_X4 = 19, OCN_OPT_CO_LAUNCH = 20, &
                                     OCN_OPT_XCHG_DELAY = 21
    integer(c_int32_t), parameter :: OCN_HALO_LOCAL = 0, OCN_HALO_SEND = 1, OCN_HALO_RECV = 2
    integer, parameter :: OCN_UNIQUE_ID_BYTES = 128   ! sizeof(ncclUniqueId)

    type, bind(C) :: ocn_block
        integer(c_int32_t) :: nx_start, nx_end, ny_start, ny_end
        integer(c_int32_t) :: bnd_x1, bnd_x2, bnd_y1, bnd_y2
        integer(c_int64_t) :: pitch
    end type

    type, bind(C) :: ocn_basin
        integer(c_int32_t) :: nx, ny
        real(c_double) :: dxst, dyst, rlon, rlat
        integer(c_int32_t) :: curve_grid
        real(c_double) :: rotation_on_lon, rotation_on_lat
    end type

    type, bind(C) :: ocn_sw_params
        integer(c_int32_t) :: full_free_surface, trans_terms, ksw_lat
        real(c_double) :: time_smooth, lvisc_2
        integer(c_int32_t) :: use_tracers, tracer_num
    end type

    type, bind(C) :: ocn_decomp
        integer(c_int32_t) :: bnx, bny, nranks, rank, device
    end type

    type, bind(C) :: ocn_block_info
        type(ocn_block) :: geom
        integer(c_int32_t) :: bm, bn
        integer(c_int32_t) :: nbr_rank(8), nbr_k(8)
    end type

    ! one copy / message of a halo exchange (ocn_halo_schedule)
    type, bind(C) :: ocn_halo_msg
        integer(c_int32_t) :: kind, peer, k, k_src, field
        integer(c_int32_t) :: dst_x0, dst_x1, dst_y0, dst_y1
        integer(c_int32_t) :: src_x0, src_x1, src_y0, src_y1
        integer(c_int32_t) :: count
        integer(c_int64_t) :: offset
    end type

    ! the transport of a context (ocn_ctx_comm_info): 0 none, 1 RCCL, 2 loopback
    type, bind(C) :: ocn_comm_info
        integer(c_int32_t) :: transport, nccl_version, comm_size, comm_rank
        integer(c_int64_t) :: exchanges, exchanges_done
        real(c_double) :: watchdog_s
    end type

    ! the x2 / x4 steps' measured overlap choice (ocn_ctx_overlap_info)
    type, bind(C) :: ocn_overlap_info
        integer(c_int32_t) :: level, state, kind, pad
        real(c_double) :: seq_ms, overlapped_ms
    end type

    ! the shader clock of the pair launches, measured in the kernel (ocn_ctx_clock_info)
    type, bind(C) :: ocn_clock_info
        integer(c_int64_t) :: launches
        real(c_double) :: clock_ghz, sampled_ms
    end type

    interface
        ! ---------------------------------------------------------------- kernel layer
        integer(c_int) function ocn_sw_update_ssh(b, tau, lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, &
                                                  vbrtr, stream) bind(C, name='ocn_sw_update_ssh')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            real(c_double), value :: tau
            type(c_ptr), value :: lu, dx, dy, dxh, dyh, hhu, hhv, sshn, sshp, ubrtr, vbrtr, stream
        end function
        integer(c_int) function ocn_hh_update(b, lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hqn, hun, &
                                              hvn, hhn, sh, h_r, stream) bind(C, name='ocn_hh_update')
            import :: c_int, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hqn, hun, hvn, hhn, sh, h_r
            type(c_ptr), value :: stream
        end function
        integer(c_int) function ocn_uv_trans_vort(b, luu, dxt, dyt, dxb, dyb, u, v, vort, stream) &
                                                  bind(C, name='ocn_uv_trans_vort')
            import :: c_int, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: luu, dxt, dyt, dxb, dyb, u, v, vort, stream
        end function
        integer(c_int) function ocn_uv_trans(b, lcu, lcv, luu, dxh, dyh, u, v, vort, hq, hu, hv, hh, rhsx, rhsy, &
                                             stream) bind(C, name='ocn_uv_trans')
            import :: c_int, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: lcu, lcv, luu, dxh, dyh, u, v, vort, hq, hu, hv, hh, rhsx, rhsy, stream
        end function
        integer(c_int) function ocn_stress_components(b, lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, &
                                                      str_t, str_s, stream) bind(C, name='ocn_stress_components')
            import :: c_int, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: lu, luu, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, u, v, str_t, str_s, stream
        end function
        integer(c_int) function ocn_uv_diff2(b, lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s, &
                                             hq, hu, hv, hh, rhsx, rhsy, stream) bind(C, name='ocn_uv_diff2')
            import :: c_int, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: lcu, lcv, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, mu, str_t, str_s
            type(c_ptr), value :: hq, hu, hv, hh, rhsx, rhsy, stream
        end function
        integer(c_int) function ocn_sw_update_uv(b, tau, lcu, lcv, dxt, dyt, dxh, dyh, dxb, dyb, hhu, hhun, hhup, &
                                                 hhv, hhvn, hhvp, hhh, ssh, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn,  &
                                                 vbrtrp, rdis, rlh_s, rhsx, rhsy, rhsx_adv, rhsy_adv, rhsx_dif,    &
                                                 rhsy_dif, stream) bind(C, name='ocn_sw_update_uv')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            real(c_double), value :: tau
            type(c_ptr), value :: lcu, lcv, dxt, dyt, dxh, dyh, dxb, dyb, hhu, hhun, hhup, hhv, hhvn, hhvp, hhh, ssh
            type(c_ptr), value :: ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp, rdis, rlh_s
            type(c_ptr), value :: rhsx, rhsy, rhsx_adv, rhsy_adv, rhsx_dif, rhsy_dif, stream
        end function
        integer(c_int) function ocn_sw_next_step(b, time_smooth, lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, &
                                                 ubrtrp, vbrtr, vbrtrn, vbrtrp, stream) bind(C, name='ocn_sw_next_step')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            real(c_double), value :: time_smooth
            type(c_ptr), value :: lu, lcu, lcv, ssh, sshn, sshp, ubrtr, ubrtrn, ubrtrp, vbrtr, vbrtrn, vbrtrp, stream
        end function
        integer(c_int) function ocn_hh_shift(b, time_smooth, lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, &
                                             hvn, hh, hhp, hhn, stream) bind(C, name='ocn_hh_shift')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            real(c_double), value :: time_smooth
            type(c_ptr), value :: lu, llu, llv, luh, hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn, stream
        end function
        integer(c_int) function ocn_hh_init(b, ffs, lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb, hq, &
                                            hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn, sh, shp, h_r, stream) &
                                            bind(C, name='ocn_hh_init')
            import :: c_int, c_int32_t, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            integer(c_int32_t), value :: ffs
            type(c_ptr), value :: lu, llu, llv, luh, dx, dy, dxt, dyt, dxh, dyh, dxb, dyb
            type(c_ptr), value :: hq, hqp, hqn, hu, hup, hun, hv, hvp, hvn, hh, hhp, hhn, sh, shp, h_r, stream
        end function

        ! ---------------------------------------------------------------- PSy layer
        integer(c_int) function ocn_ctx_create(basin, sw, dec, mask, ctx) bind(C, name='ocn_ctx_create')
            import :: c_int, c_ptr, ocn_basin, ocn_sw_params, ocn_decomp
            type(ocn_basin), intent(in) :: basin
            type(ocn_sw_params), intent(in) :: sw
            type(ocn_decomp), intent(in) :: dec
            type(c_ptr), value :: mask
            type(c_ptr), intent(out) :: ctx
        end function
        integer(c_int) function ocn_ctx_destroy(ctx) bind(C, name='ocn_ctx_destroy')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        integer(c_int) function ocn_ctx_block_count(ctx) bind(C, name='ocn_ctx_block_count')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        integer(c_int) function ocn_ctx_block_info(ctx, k, info) bind(C, name='ocn_ctx_block_info')
            import :: c_int, c_ptr, ocn_block_info
            type(c_ptr), value :: ctx
            integer(c_int), value :: k
            type(ocn_block_info), intent(out) :: info
        end function
        type(c_ptr) function ocn_ctx_field(ctx, k, id) bind(C, name='ocn_ctx_field')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: k, id
        end function
        type(c_ptr) function ocn_ctx_stream(ctx) bind(C, name='ocn_ctx_stream')
            import :: c_ptr
            type(c_ptr), value :: ctx
        end function
        ! control/init_data.f90:115-120: the basin.par topography file's real(4) interior values
        integer(c_int) function ocn_ctx_set_topography(ctx, h, count) bind(C, name='ocn_ctx_set_topography')
            import :: c_int, c_int64_t, c_ptr
            type(c_ptr), value :: ctx, h
            integer(c_int64_t), value :: count
        end function
        integer(c_int) function ocn_ctx_init_state(ctx) bind(C, name='ocn_ctx_init_state')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        ! forms a pending call tail (OCN_OPT_LAZY_TAIL) before a host reads device memory itself
        integer(c_int) function ocn_ctx_complete(ctx) bind(C, name='ocn_ctx_complete')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        integer(c_int) function ocn_ctx_sync(ctx, id) bind(C, name='ocn_ctx_sync')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: id
        end function
        integer(c_int) function ocn_ctx_stage(ctx, stage, tau) bind(C, name='ocn_ctx_stage')
            import :: c_int, c_double, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: stage
            real(c_double), value :: tau
        end function
        integer(c_int) function ocn_ctx_step(ctx, tau, nsteps, check_every) bind(C, name='ocn_ctx_step')
            import :: c_int, c_int32_t, c_double, c_ptr
            type(c_ptr), value :: ctx
            real(c_double), value :: tau
            integer(c_int32_t), value :: nsteps, check_every
        end function
        integer(c_int) function ocn_ctx_synchronize(ctx) bind(C, name='ocn_ctx_synchronize')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
        end function
        integer(c_int) function ocn_ctx_download(ctx, k, id, host) bind(C, name='ocn_ctx_download')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: k, id
            type(c_ptr), value :: host
        end function
        ! output.f90 copy_from_real8 + io.f90 write_data2D_real4: interior record as real(4), undef on land
        integer(c_int) function ocn_ctx_output_r4(ctx, k, id, undef, host) bind(C, name='ocn_ctx_output_r4')
            import :: c_int, c_ptr, c_float
            type(c_ptr), value :: ctx
            integer(c_int), value :: k, id
            real(c_float), value :: undef
            type(c_ptr), value :: host
        end function
        integer(c_int) function ocn_ctx_upload(ctx, k, id, host) bind(C, name='ocn_ctx_upload')
            import :: c_int, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: k, id
            type(c_ptr), value :: host
        end function
        integer(c_int) function ocn_ctx_set_option(ctx, key, val) bind(C, name='ocn_ctx_set_option')
            import :: c_int, c_int32_t, c_int64_t, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int32_t), value :: key
            integer(c_int64_t), value :: val
        end function
        integer(c_int) function ocn_ctx_get_option(ctx, key, val) bind(C, name='ocn_ctx_get_option')
            import :: c_int, c_int32_t, c_int64_t, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int32_t), value :: key
            integer(c_int64_t), intent(out) :: val
        end function
        ! ---------------------------------------------------------------- ranks (shared/mpp/mpp.f90:64-221)
        ! host-only: the blocks rank dec%rank owns (core/decomposition.f90:614-669), and one exchange's
        ! copies / messages (shared/mpp/syncborder_block2D_gen_all.fi)
        integer(c_int) function ocn_decompose(basin, dec, mask, out, cap, count) bind(C, name='ocn_decompose')
            import :: c_int, c_int32_t, c_ptr, ocn_basin, ocn_decomp
            type(ocn_basin), intent(in) :: basin
            type(ocn_decomp), intent(in) :: dec
            type(c_ptr), value :: mask, out
            integer(c_int32_t), value :: cap
            integer(c_int32_t), intent(out) :: count
        end function
        integer(c_int) function ocn_halo_schedule(basin, dec, mask, field_ids, nfields, out, cap, count) &
                                                  bind(C, name='ocn_halo_schedule')
            import :: c_int, c_int32_t, c_ptr, ocn_basin, ocn_decomp
            type(ocn_basin), intent(in) :: basin
            type(ocn_decomp), intent(in) :: dec
            type(c_ptr), value :: mask, field_ids
            integer(c_int32_t), value :: nfields
            type(c_ptr), value :: out
            integer(c_int32_t), value :: cap
            integer(c_int32_t), intent(out) :: count
        end function
        ! RCCL: rank 0 makes the unique id (128 bytes), the host hands it to every rank, each attaches
        integer(c_int) function ocn_comm_unique_id(out_id, nbytes) bind(C, name='ocn_comm_unique_id')
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value :: out_id
            integer(c_int32_t), value :: nbytes
        end function
        integer(c_int) function ocn_ctx_attach_comm(ctx, unique_id, nbytes) bind(C, name='ocn_ctx_attach_comm')
            import :: c_int, c_int32_t, c_ptr
            type(c_ptr), value :: ctx, unique_id
            integer(c_int32_t), value :: nbytes
        end function
        integer(c_int) function ocn_ctx_comm_info(ctx, info) bind(C, name='ocn_ctx_comm_info')
            import :: c_int, c_ptr, ocn_comm_info
            type(c_ptr), value :: ctx
            type(ocn_comm_info), intent(out) :: info
        end function
        integer(c_int) function ocn_ctx_overlap_info(ctx, info) bind(C, name='ocn_ctx_overlap_info')
            import :: c_int, c_ptr, ocn_overlap_info
            type(c_ptr), value :: ctx
            type(ocn_overlap_info), intent(out) :: info
        end function
        integer(c_int) function ocn_ctx_clock_info(ctx, reset, info) bind(C, name='ocn_ctx_clock_info')
            import :: c_int, c_int32_t, c_ptr, ocn_clock_info
            type(c_ptr), value :: ctx
            integer(c_int32_t), value :: reset
            type(ocn_clock_info), intent(out) :: info
        end function
        integer(c_int) function ocn_ctx_set_watchdog(ctx, seconds) bind(C, name='ocn_ctx_set_watchdog')
            import :: c_int, c_double, c_ptr
            type(c_ptr), value :: ctx
            real(c_double), value :: seconds
        end function
        type(c_ptr) function ocn_last_error() bind(C, name='ocn_last_error')
            import :: c_ptr
        end function
        ! kernel/tracer/leapfrog_tracer.f90:13, :94, :138
        integer(c_int) function ocn_tran_diff_fluxes(b, lcu, lcv, dxt, dyt, dxh, dyh, hhu, hhv, ff, ffp, uu, vv, &
                                                     mu, factor_mu, flux_x, flux_y, stream)                    &
                                                     bind(C, name='ocn_tran_diff_fluxes')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: lcu, lcv, dxt, dyt, dxh, dyh, hhu, hhv, ff, ffp, uu, vv, mu
            real(c_double), value :: factor_mu
            type(c_ptr), value :: flux_x, flux_y, stream
        end function
        integer(c_int) function ocn_tran_diff_tracer(b, lu, dx, dy, tau, hhqn, hhqp, flux_x, flux_y, ffp, ffn,  &
                                                     stream) bind(C, name='ocn_tran_diff_tracer')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            type(c_ptr), value :: lu, dx, dy
            real(c_double), value :: tau
            type(c_ptr), value :: hhqn, hhqp, flux_x, flux_y, ffp, ffn, stream
        end function
        integer(c_int) function ocn_tracer_next_step(b, time_smooth, lu, ffn, ffp, ff, stream) &
                                                     bind(C, name='ocn_tracer_next_step')
            import :: c_int, c_double, c_ptr, ocn_block
            type(ocn_block), intent(in) :: b
            real(c_double), value :: time_smooth
            type(c_ptr), value :: lu, ffn, ffp, ff, stream
        end function
        integer(c_int) function ocn_ctx_tracer_stage(ctx, stage, tracer, tau) bind(C, name='ocn_ctx_tracer_stage')
            import :: c_int, c_double, c_ptr
            type(c_ptr), value :: ctx
            integer(c_int), value :: stage, tracer
            real(c_double), value :: tau
        end function
    end interface

contains

    subroutine ocn_check(rc, what)
        integer(c_int), intent(in) :: rc
        character(*), intent(in) :: what
        character(kind=c_char), pointer :: msg(:)
        integer :: i
        if (rc == OCN_OK) return
        call c_f_pointer(ocn_last_error(), msg, [512])
        write(*, '(a,a,i0,a)', advance='no') what, ': ocn error ', rc, ': '
        do i = 1, 512
            if (msg(i) == c_null_char) exit
            write(*, '(a)', advance='no') msg(i)
        enddo
        write(*, *)
        error stop 2
    end subroutine

end module ocn_sw_c
