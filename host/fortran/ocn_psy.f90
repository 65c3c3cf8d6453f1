! ocn_psy.f90 -- Fortran PSy + Algorithm layers over libocn_sw (ISO_C_BINDING).
!
! Same shape as the reference: kernel_parameters_type + envoke(sub_kernel, sub_sync, params)
! (core/kernel_interface.f90:15-119), envoke_<stage>_kernel / envoke_<stage>_sync wrappers that
! hand block k's device fields to the kernel (interface/shallow_water/sw_interface.f90), and
! expl_shallow_water(tau) (control/shallow_water/shallow_water.f90:22-94).  The difference from
! the reference: the field "block(k)%field" is a device address owned by libocn_sw, and the
! kernel is an extern "C" HIP entry instead of a Fortran loop nest.
module ocn_psy
    use iso_c_binding
    use ocn_sw_c
    implicit none
    private

    type, public :: kernel_parameters_type
        real(c_double) :: tau = 0.0d0
        real(c_double) :: time_smooth = 0.0d0
        integer :: data_id = 0
    contains
        procedure, public :: clear => clear_kernel_parameters
    end type

    type, public :: sync_parameters_type
        integer :: sync_mode = 3
        integer :: data_id = 0
    end type

    abstract interface
        subroutine envoke_kernel_iface(k, param)
            import :: kernel_parameters_type
            integer, intent(in) :: k
            type(kernel_parameters_type), intent(in) :: param
        end subroutine
        subroutine envoke_sync_iface(k, sp)
            import :: sync_parameters_type
            integer, intent(in) :: k
            type(sync_parameters_type), intent(in) :: sp
        end subroutine
    end interface

    ! model state of this process (the reference's domain_data / ocean_data / grid_data)
    type(c_ptr), public :: ctx = c_null_ptr
    integer, public :: bcount = 0
    type(ocn_block), allocatable, public :: blk(:)
    type(ocn_sw_params), public :: sw_params
    ! psy_fused (default): expl_shallow_water is one ocn_ctx_step(ctx, tau, 1) -- the library's fused
    ! step, expl_tracer included (model.f90:146-160), which continues a one-pass sequence across
    ! calls (OCN_OPT_LAZY_TAIL); .false.: the reference's 11 envoke stages through the kernel-layer
    ! entries (per-stage hooks, e.g. to inspect a stage's output).  Same results bit for bit.
    logical, public :: psy_fused = .true.

    public :: psy_init, envoke, expl_shallow_water, expl_tracer, fld

contains

    subroutine clear_kernel_parameters(this)
        class(kernel_parameters_type), intent(inout) :: this
        this%tau = 0.0d0; this%time_smooth = 0.0d0; this%data_id = 0
    end subroutine

    subroutine psy_init(c, sw)
        type(c_ptr), intent(in) :: c
        type(ocn_sw_params), intent(in) :: sw
        type(ocn_block_info) :: info
        integer :: k
        ctx = c
        sw_params = sw
        bcount = ocn_ctx_block_count(ctx)
        allocate(blk(bcount))
        do k = 1, bcount
            call ocn_check(ocn_ctx_block_info(ctx, k - 1, info), 'ocn_ctx_block_info')
            blk(k) = info%geom
        enddo
    end subroutine

    type(c_ptr) function fld(k, id)
        integer, intent(in) :: k
        integer(c_int), intent(in) :: id
        fld = ocn_ctx_field(ctx, int(k - 1, c_int), id)
    end function

    ! core/kernel_interface.f90:48-119 (_MPP_NO_PARALLEL_MODE_ path)
    subroutine envoke(sub_kernel, sub_sync, param)
        procedure(envoke_kernel_iface) :: sub_kernel
        procedure(envoke_sync_iface) :: sub_sync
        type(kernel_parameters_type), intent(in) :: param
        type(sync_parameters_type) :: sp
        integer :: k
        do k = 1, bcount
            call sub_kernel(k, param)
        enddo
        sp%sync_mode = 3
        sp%data_id = param%data_id
        call sub_sync(-1, sp)
    end subroutine

    ! ------------------------------------------------------------- per-kernel wrappers
    subroutine envoke_sw_update_ssh_kernel(k, param)       ! sw_interface.f90:310
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_sw_update_ssh(blk(k), param%tau, fld(k, OCN_LU), fld(k, OCN_DX), fld(k, OCN_DY), &
                       fld(k, OCN_DXH), fld(k, OCN_DYH), fld(k, OCN_HHU), fld(k, OCN_HHV), fld(k, OCN_SSHN),     &
                       fld(k, OCN_SSHP), fld(k, OCN_UBRTR), fld(k, OCN_VBRTR), ocn_ctx_stream(ctx)), 'sw_update_ssh')
    end subroutine
    subroutine envoke_sw_update_ssh_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_SSHN), 'sync sshn')
    end subroutine

    subroutine envoke_hh_update_kernel(k, param)           ! sw_interface.f90:145
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_hh_update(blk(k), fld(k, OCN_LU), fld(k, OCN_LLU), fld(k, OCN_LLV), fld(k, OCN_LUH), &
                       fld(k, OCN_DX), fld(k, OCN_DY), fld(k, OCN_DXT), fld(k, OCN_DYT), fld(k, OCN_DXH),         &
                       fld(k, OCN_DYH), fld(k, OCN_DXB), fld(k, OCN_DYB), fld(k, OCN_HHQ_N), fld(k, OCN_HHU_N),   &
                       fld(k, OCN_HHV_N), fld(k, OCN_HHH_N), fld(k, OCN_SSH), fld(k, OCN_HHQ_REST),              &
                       ocn_ctx_stream(ctx)), 'hh_update')
    end subroutine
    subroutine envoke_hh_update_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_HHU_N), 'sync'); call ocn_check(ocn_ctx_sync(ctx, OCN_HHV_N), 'sync')
        call ocn_check(ocn_ctx_sync(ctx, OCN_HHH_N), 'sync')
    end subroutine

    subroutine envoke_uv_trans_vort_kernel(k, param)       ! sw_interface.f90:211
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_uv_trans_vort(blk(k), fld(k, OCN_LUU), fld(k, OCN_DXT), fld(k, OCN_DYT), fld(k, OCN_DXB), &
                       fld(k, OCN_DYB), fld(k, OCN_UBRTR), fld(k, OCN_VBRTR), fld(k, OCN_VORT), ocn_ctx_stream(ctx)), &
                       'uv_trans_vort')
    end subroutine
    subroutine envoke_uv_trans_vort_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_VORT), 'sync vort')
    end subroutine

    subroutine envoke_uv_trans_kernel(k, param)            ! sw_interface.f90:238
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_uv_trans(blk(k), fld(k, OCN_LCU), fld(k, OCN_LCV), fld(k, OCN_LUU), fld(k, OCN_DXH),    &
                       fld(k, OCN_DYH), fld(k, OCN_UBRTR), fld(k, OCN_VBRTR), fld(k, OCN_VORT), fld(k, OCN_HHQ),      &
                       fld(k, OCN_HHU), fld(k, OCN_HHV), fld(k, OCN_HHH), fld(k, OCN_RHSX_ADV), fld(k, OCN_RHSY_ADV), &
                       ocn_ctx_stream(ctx)), 'uv_trans')
    end subroutine
    subroutine envoke_uv_trans_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_HHU_P), 'sync'); call ocn_check(ocn_ctx_sync(ctx, OCN_HHV_P), 'sync')
        call ocn_check(ocn_ctx_sync(ctx, OCN_HHH_P), 'sync')
    end subroutine

    subroutine envoke_stress_components_kernel(k, param)   ! sw_interface.f90:110
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_stress_components(blk(k), fld(k, OCN_LU), fld(k, OCN_LUU), fld(k, OCN_DX), fld(k, OCN_DY), &
                       fld(k, OCN_DXT), fld(k, OCN_DYT), fld(k, OCN_DXH), fld(k, OCN_DYH), fld(k, OCN_DXB),            &
                       fld(k, OCN_DYB), fld(k, OCN_UBRTRP), fld(k, OCN_VBRTRP), fld(k, OCN_STR_T), fld(k, OCN_STR_S),   &
                       ocn_ctx_stream(ctx)), 'stress_components')
    end subroutine
    subroutine envoke_stress_components_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_STR_T), 'sync'); call ocn_check(ocn_ctx_sync(ctx, OCN_STR_S), 'sync')
    end subroutine

    subroutine envoke_uv_diff2_kernel(k, param)            ! sw_interface.f90:273
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_uv_diff2(blk(k), fld(k, OCN_LCU), fld(k, OCN_LCV), fld(k, OCN_DX), fld(k, OCN_DY),     &
                       fld(k, OCN_DXT), fld(k, OCN_DYT), fld(k, OCN_DXH), fld(k, OCN_DYH), fld(k, OCN_DXB),        &
                       fld(k, OCN_DYB), fld(k, OCN_MU), fld(k, OCN_STR_T), fld(k, OCN_STR_S), fld(k, OCN_HHQ),     &
                       fld(k, OCN_HHU), fld(k, OCN_HHV), fld(k, OCN_HHH), fld(k, OCN_RHSX_DIF), fld(k, OCN_RHSY_DIF), &
                       ocn_ctx_stream(ctx)), 'uv_diff2')
    end subroutine

    subroutine envoke_sw_update_uv_kernel(k, param)        ! sw_interface.f90:337
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_sw_update_uv(blk(k), param%tau, fld(k, OCN_LCU), fld(k, OCN_LCV), fld(k, OCN_DXT),     &
                       fld(k, OCN_DYT), fld(k, OCN_DXH), fld(k, OCN_DYH), fld(k, OCN_DXB), fld(k, OCN_DYB),         &
                       fld(k, OCN_HHU), fld(k, OCN_HHU_N), fld(k, OCN_HHU_P), fld(k, OCN_HHV), fld(k, OCN_HHV_N),   &
                       fld(k, OCN_HHV_P), fld(k, OCN_HHH), fld(k, OCN_SSH), fld(k, OCN_UBRTR), fld(k, OCN_UBRTRN),  &
                       fld(k, OCN_UBRTRP), fld(k, OCN_VBRTR), fld(k, OCN_VBRTRN), fld(k, OCN_VBRTRP),              &
                       fld(k, OCN_R_DISS), fld(k, OCN_RLH_S), fld(k, OCN_RHSX), fld(k, OCN_RHSY),                   &
                       fld(k, OCN_RHSX_ADV), fld(k, OCN_RHSY_ADV), fld(k, OCN_RHSX_DIF), fld(k, OCN_RHSY_DIF),      &
                       ocn_ctx_stream(ctx)), 'sw_update_uv')
    end subroutine
    subroutine envoke_sw_update_uv_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_VBRTRN), 'sync'); call ocn_check(ocn_ctx_sync(ctx, OCN_UBRTRN), 'sync')
    end subroutine

    subroutine envoke_sw_next_step_kernel(k, param)        ! sw_interface.f90:384
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_sw_next_step(blk(k), param%time_smooth, fld(k, OCN_LU), fld(k, OCN_LCU), fld(k, OCN_LCV), &
                       fld(k, OCN_SSH), fld(k, OCN_SSHN), fld(k, OCN_SSHP), fld(k, OCN_UBRTR), fld(k, OCN_UBRTRN),     &
                       fld(k, OCN_UBRTRP), fld(k, OCN_VBRTR), fld(k, OCN_VBRTRN), fld(k, OCN_VBRTRP),                 &
                       ocn_ctx_stream(ctx)), 'sw_next_step')
    end subroutine

    subroutine envoke_hh_shift_kernel(k, param)            ! sw_interface.f90:181
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_hh_shift(blk(k), sw_params%time_smooth, fld(k, OCN_LU), fld(k, OCN_LLU), fld(k, OCN_LLV), &
                       fld(k, OCN_LUH), fld(k, OCN_HHQ), fld(k, OCN_HHQ_P), fld(k, OCN_HHQ_N), fld(k, OCN_HHU),       &
                       fld(k, OCN_HHU_P), fld(k, OCN_HHU_N), fld(k, OCN_HHV), fld(k, OCN_HHV_P), fld(k, OCN_HHV_N),    &
                       fld(k, OCN_HHH), fld(k, OCN_HHH_P), fld(k, OCN_HHH_N), ocn_ctx_stream(ctx)), 'hh_shift')
    end subroutine

    subroutine envoke_hh_init_kernel(k, param)             ! sw_interface.f90:42
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        call ocn_check(ocn_hh_init(blk(k), sw_params%full_free_surface, fld(k, OCN_LU), fld(k, OCN_LLU),           &
                       fld(k, OCN_LLV), fld(k, OCN_LUH), fld(k, OCN_DX), fld(k, OCN_DY), fld(k, OCN_DXT),           &
                       fld(k, OCN_DYT), fld(k, OCN_DXH), fld(k, OCN_DYH), fld(k, OCN_DXB), fld(k, OCN_DYB),         &
                       fld(k, OCN_HHQ), fld(k, OCN_HHQ_P), fld(k, OCN_HHQ_N), fld(k, OCN_HHU), fld(k, OCN_HHU_P),   &
                       fld(k, OCN_HHU_N), fld(k, OCN_HHV), fld(k, OCN_HHV_P), fld(k, OCN_HHV_N), fld(k, OCN_HHH),   &
                       fld(k, OCN_HHH_P), fld(k, OCN_HHH_N), fld(k, OCN_SSH), fld(k, OCN_SSHP), fld(k, OCN_HHQ_REST), &
                       ocn_ctx_stream(ctx)), 'hh_init')
    end subroutine
    subroutine envoke_hh_init_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_HHU), 'sync'); call ocn_check(ocn_ctx_sync(ctx, OCN_HHV), 'sync')
        call ocn_check(ocn_ctx_sync(ctx, OCN_HHH), 'sync')
    end subroutine

    subroutine envoke_empty_sync(k, sp)                    ! kernel_interface.f90:43
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
    end subroutine

    ! ------------------------------------------------------------- tracer wrappers
    ! interface/tracer/tracer_interface.f90 (tracer = param%data_id)
    subroutine envoke_tran_diff_fluxes_kernel(k, param)    ! tracer_interface.f90:28
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        integer(c_int) :: t
        t = OCN_TRACER_BASE + 3 * (param%data_id - 1)
        call ocn_check(ocn_tran_diff_fluxes(blk(k), fld(k, OCN_LCU), fld(k, OCN_LCV), fld(k, OCN_DXT),          &
                       fld(k, OCN_DYT), fld(k, OCN_DXH), fld(k, OCN_DYH), fld(k, OCN_HHU), fld(k, OCN_HHV),       &
                       fld(k, t), fld(k, t + 1), fld(k, OCN_UBRTR), fld(k, OCN_VBRTR), fld(k, OCN_MU), 1.0d0,    &
                       fld(k, OCN_FLUX_X), fld(k, OCN_FLUX_Y), ocn_ctx_stream(ctx)), 'tran_diff_fluxes')
    end subroutine
    subroutine envoke_tran_diff_fluxes_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, OCN_FLUX_X), 'sync'); call ocn_check(ocn_ctx_sync(ctx, OCN_FLUX_Y), 'sync')
    end subroutine

    subroutine envoke_tran_diff_tracer_kernel(k, param)    ! tracer_interface.f90:61
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        integer(c_int) :: t
        t = OCN_TRACER_BASE + 3 * (param%data_id - 1)
        call ocn_check(ocn_tran_diff_tracer(blk(k), fld(k, OCN_LU), fld(k, OCN_DX), fld(k, OCN_DY), param%tau,   &
                       fld(k, OCN_HHQ_N), fld(k, OCN_HHQ_P), fld(k, OCN_FLUX_X), fld(k, OCN_FLUX_Y),             &
                       fld(k, t + 1), fld(k, t + 2), ocn_ctx_stream(ctx)), 'tran_diff_tracer')
    end subroutine
    subroutine envoke_tran_diff_tracer_sync(k, sp)
        integer, intent(in) :: k
        type(sync_parameters_type), intent(in) :: sp
        call ocn_check(ocn_ctx_sync(ctx, int(OCN_TRACER_BASE + 3 * (sp%data_id - 1) + 2, c_int)), 'sync ff1n')
    end subroutine

    subroutine envoke_tracer_next_step_kernel(k, param)    ! tracer_interface.f90:88
        integer, intent(in) :: k
        type(kernel_parameters_type), intent(in) :: param
        integer(c_int) :: t
        t = OCN_TRACER_BASE + 3 * (param%data_id - 1)
        call ocn_check(ocn_tracer_next_step(blk(k), param%time_smooth, fld(k, OCN_LU), fld(k, t + 2),             &
                       fld(k, t + 1), fld(k, t), ocn_ctx_stream(ctx)), 'tracer_next_step')
    end subroutine

    ! ------------------------------------------------------------- algorithm layer
    ! control/tracer.f90:33-62
    subroutine expl_tracer(tau)
        real(c_double), intent(in) :: tau
        type(kernel_parameters_type) :: p
        integer :: k
        if (sw_params%use_tracers <= 0) return
        if (psy_fused) return   ! ran inside expl_shallow_water's ocn_ctx_step
        do k = 1, sw_params%tracer_num
            call p%clear()
            p%tau = tau
            p%time_smooth = sw_params%time_smooth
            p%data_id = k
            call envoke(envoke_tran_diff_fluxes_kernel, envoke_tran_diff_fluxes_sync, p)
            call envoke(envoke_tran_diff_tracer_kernel, envoke_tran_diff_tracer_sync, p)
            call envoke(envoke_tracer_next_step_kernel, envoke_empty_sync, p)
        enddo
    end subroutine

    ! control/shallow_water/shallow_water.f90:22-94
    subroutine expl_shallow_water(tau)
        real(c_double), intent(in) :: tau
        type(kernel_parameters_type) :: p
        if (psy_fused) then
            call ocn_check(ocn_ctx_step(ctx, tau, 1_c_int32_t, 1_c_int32_t), 'ocn_ctx_step')
            return
        endif
        call p%clear()
        p%tau = tau
        p%time_smooth = sw_params%time_smooth

        call envoke(envoke_sw_update_ssh_kernel, envoke_sw_update_ssh_sync, p)
        if (sw_params%full_free_surface > 0) call envoke(envoke_hh_update_kernel, envoke_hh_update_sync, p)
        if (sw_params%trans_terms > 0) then
            call envoke(envoke_uv_trans_vort_kernel, envoke_uv_trans_vort_sync, p)
            call envoke(envoke_uv_trans_kernel, envoke_uv_trans_sync, p)
        endif
        if (sw_params%ksw_lat > 0) then
            call envoke(envoke_stress_components_kernel, envoke_stress_components_sync, p)
            call envoke(envoke_uv_diff2_kernel, envoke_empty_sync, p)
        endif
        call envoke(envoke_sw_update_uv_kernel, envoke_sw_update_uv_sync, p)
        call envoke(envoke_sw_next_step_kernel, envoke_empty_sync, p)
        if (sw_params%full_free_surface > 0) then
            call envoke(envoke_hh_shift_kernel, envoke_empty_sync, p)
            call envoke(envoke_hh_init_kernel, envoke_hh_init_sync, p)
        endif
        ! check_ssh_err (vel_ssh.f90:40) as a device reduction, reported at synchronize
        call ocn_check(ocn_ctx_stage(ctx, OCN_STAGE_CHECK_SSH_ERR, tau), 'check_ssh_err')
    end subroutine

end module ocn_psy
