! ocn_sw_driver.f90 -- Fortran host program: the reference's model.f90 time loop with the
! shallow-water step running on the MI355X through libocn_sw.
!
! usage (in a directory holding basin.par, sw.par, parallel.par):
!     ocn_sw_driver NSTEPS DUMPFILE [native|stages]
!     ocn_sw_driver plan PLANFILE      (host only, no GPU: this rank's blocks + schedule -> PLANFILE.r<rank>)
! Reads the positional .par files (first lexeme per line, readpar semantics), builds the model
! (decomposition + init_grid_data + init_ocean_data on the device), runs NSTEPS of
! expl_shallow_water + expl_tracer through the Fortran PSy layer -- by default its fused form (one
! ocn_ctx_step per time step), with "stages" the reference's envoke stages, with "native" one
! ocn_ctx_step call of NSTEPS -- and writes every field of every block in the oracle/ref_driver.f90
! dump format.
!
! Ranks (shared/mpp/mpp.f90:64-221 mpp_init): one process per GPU.  Built with MPI (make MPI=1:
! ocn_sw_driver_mpi, -DOCN_MPI) the rank and the rank count come from mpi_comm_rank /
! mpi_comm_size on MPI_COMM_WORLD and rank 0's RCCL unique id reaches the others by mpi_bcast;
! without MPI from RANK / WORLD_SIZE / LOCAL_RANK (torch.distributed.run's variables) and a file
! rank 0 writes (OCN_UID_FILE).  The device is LOCAL_RANK (MPI: OCN_DEVICE, else 0).  The blocks a
! rank owns are dealt by the library exactly as create_uniform_decomposition deals them over the
! mpi_dims_create process grid (core/decomposition.f90:614-669, mpp.f90:89).  With more than one
! rank -- or OCN_ATTACH_COMM=1 for a one-rank communicator -- an RCCL communicator carries the halo
! exchanges (ocn_ctx_attach_comm); OCN_WATCHDOG=<seconds> arms the library's watchdog.  Each rank
! writes DUMPFILE (one rank) or DUMPFILE.r<rank>.
program ocn_sw_driver
    use iso_c_binding
    use ocn_sw_c
    use ocn_psy
#ifdef OCN_MPI
    use mpi
#endif
    implicit none

    interface   ! libc
        integer(c_int) function c_rename(old, new) bind(C, name='rename')
            import :: c_int, c_char
            character(kind=c_char), intent(in) :: old(*), new(*)
        end function
        integer(c_int) function c_usleep(us) bind(C, name='usleep')
            import :: c_int
            integer(c_int), value :: us
        end function
    end interface

    integer :: nsteps, step, k, id, u, nx, ny, nlo, ntr, rank, nranks, local_rank
    character(len=512) :: arg, dumpfile, maskfile, topofile, env
    character(len=256) :: lines(32)
    type(ocn_basin) :: basin
    type(ocn_sw_params) :: sw
    type(ocn_decomp) :: dec
    type(ocn_block_info) :: info
    type(c_ptr) :: c
    integer(c_int32_t), allocatable, target :: mask(:, :)
    real(c_float), allocatable, target :: a4(:, :)
    real(c_double), allocatable, target :: a8(:, :)
    real(c_float), allocatable, target :: topo(:, :)
    character(kind=c_char), target :: uid(OCN_UNIQUE_ID_BYTES)
    logical :: native, plan, attach
    real(c_double) :: wd
    integer, parameter :: r4_order(17) = [0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16]
#ifdef OCN_MPI
    integer :: ierr
#endif

    call get_command_argument(1, arg)
    plan = trim(arg) == 'plan'
    if (.not. plan) read(arg, *) nsteps
    call get_command_argument(2, dumpfile)
    call get_command_argument(3, arg); native = (trim(arg) == 'native')
    if (trim(arg) == 'stages') psy_fused = .false.

    call ranks_init(rank, nranks, local_rank)

    ! basin.par (configs/basinpar.f90:53-77)
    call read_par('basin.par', lines, nlo)
    read(lines(1), *) basin%nx; read(lines(2), *) basin%ny
    read(lines(6), *) basin%dxst; read(lines(7), *) basin%dyst
    read(lines(8), *) basin%rlon; read(lines(9), *) basin%rlat
    read(lines(12), *) basin%curve_grid
    read(lines(13), *) basin%rotation_on_lon; read(lines(14), *) basin%rotation_on_lat
    maskfile = lines(19)
    topofile = lines(20)
    ! sw.par (configs/sw.f90:34-41)
    call read_par('sw.par', lines, nlo)
    read(lines(1), *) sw%full_free_surface; read(lines(2), *) sw%trans_terms; read(lines(3), *) sw%ksw_lat
    read(lines(4), *) sw%time_smooth; read(lines(5), *) sw%lvisc_2
    read(lines(6), *) sw%use_tracers; read(lines(7), *) sw%tracer_num
    ! parallel.par (configs/parallel.f90:34-37), _DD_MANUAL_BLOCK_GRID_: the block grid; the blocks are
    ! dealt to the nranks processes (create_uniform_decomposition)
    call read_par('parallel.par', lines, nlo)
    read(lines(3), *) dec%bnx; read(lines(4), *) dec%bny
    dec%nranks = nranks; dec%rank = rank; dec%device = local_rank

    nx = basin%nx; ny = basin%ny
    if (trim(maskfile) /= 'none') then
        allocate(mask(nx, ny))
        call read_mask(trim(maskfile), nx, ny, mask)
    endif
    if (plan) then   ! PLANFILE.r<rank>
        write(dumpfile, '(a,a,i0)') trim(dumpfile), '.r', rank
        call write_plan(trim(dumpfile))
    else
        call run_model()
    endif
    call ranks_finalize()

contains

    ! the model on this rank's blocks: create, communicator, init, the time loop, the dump
    subroutine run_model()
        if (allocated(mask)) then
            call ocn_check(ocn_ctx_create(basin, sw, dec, c_loc(mask), c), 'ocn_ctx_create')
        else
            call ocn_check(ocn_ctx_create(basin, sw, dec, c_null_ptr, c), 'ocn_ctx_create')
        endif
        call get_environment_variable('OCN_ATTACH_COMM', env)
        attach = nranks > 1 .or. trim(env) == '1'
        if (attach) then   ! RCCL (mpp_init's communicator): rank 0's unique id, then every rank attaches
            call share_unique_id()
            call ocn_check(ocn_ctx_attach_comm(c, c_loc(uid), int(OCN_UNIQUE_ID_BYTES, c_int32_t)), 'ocn_ctx_attach_comm')
        endif
        call get_environment_variable('OCN_WATCHDOG', env)
        if (len_trim(env) > 0) then
            read(env, *) wd
            call ocn_check(ocn_ctx_set_watchdog(c, wd), 'ocn_ctx_set_watchdog')
        endif
        call psy_init(c, sw)
        if (len_trim(topofile) > 0 .and. trim(topofile) /= 'none') then   ! init_data.f90:115-120
            allocate(topo(nx - 4, ny - 4))
            open(newunit=u, file=trim(topofile), access='stream', form='unformatted', status='old', action='read')
            read(u) topo
            close(u)
            call ocn_check(ocn_ctx_set_topography(c, c_loc(topo), int(size(topo), c_int64_t)), 'set_topography')
        endif
        call ocn_check(ocn_ctx_init_state(c), 'ocn_ctx_init_state')

        if (native) then
            call ocn_check(ocn_ctx_step(c, 1.0d0, int(nsteps, c_int32_t), 1_c_int32_t), 'ocn_ctx_step')
        else
            do step = 1, nsteps                       ! model.f90:146-160
                call expl_shallow_water(1.0d0)
                call expl_tracer(1.0d0)
            enddo
        endif
        call ocn_check(ocn_ctx_synchronize(c), 'ocn_ctx_synchronize')   ! (every rank: a collective)

        if (nranks > 1) write(dumpfile, '(a,a,i0)') trim(dumpfile), '.r', rank
        open(newunit=u, file=trim(dumpfile), access='stream', form='unformatted', status='replace')
        ntr = 0
        if (sw%use_tracers > 0) ntr = sw%tracer_num
        write(u) int(bcount, c_int32_t), int(ntr, c_int32_t)
        do k = 1, bcount
            call ocn_check(ocn_ctx_block_info(c, int(k - 1, c_int), info), 'block_info')
            write(u) info%bm, info%bn, info%geom%nx_start, info%geom%nx_end, info%geom%ny_start, info%geom%ny_end, &
                     info%geom%bnd_x1, info%geom%bnd_x2, info%geom%bnd_y1, info%geom%bnd_y2
            allocate(a4(info%geom%bnd_x1:info%geom%bnd_x2, info%geom%bnd_y1:info%geom%bnd_y2))
            allocate(a8(info%geom%bnd_x1:info%geom%bnd_x2, info%geom%bnd_y1:info%geom%bnd_y2))
            do id = 1, 17
                call ocn_check(ocn_ctx_download(c, int(k - 1, c_int), int(r4_order(id), c_int), c_loc(a4)), 'download')
                write(u) a4
            enddo
            do id = OCN_SSH, OCN_FIELD_END - 1 + merge(2 + 3 * ntr, 0, ntr > 0)   ! + flux_x, flux_y, ff1/ff1p/ff1n
                call ocn_check(ocn_ctx_download(c, int(k - 1, c_int), int(id, c_int), c_loc(a8)), 'download')
                write(u) a8
            enddo
            deallocate(a4, a8)
        enddo
        close(u)
        call ocn_check(ocn_ctx_destroy(c), 'ocn_ctx_destroy')
    end subroutine

    ! mpp_init (shared/mpp/mpp.f90:64-221): this process's rank, the rank count, its device
    subroutine ranks_init(r, n, dev)
        integer, intent(out) :: r, n, dev
        character(len=64) :: v
        integer :: st
#ifdef OCN_MPI
        call mpi_init(ierr)
        call mpi_comm_rank(MPI_COMM_WORLD, r, ierr)
        call mpi_comm_size(MPI_COMM_WORLD, n, ierr)
        dev = 0
        call get_environment_variable('OCN_DEVICE', v, status=st)
        if (st == 0) read(v, *) dev
#else
        r = 0; n = 1; dev = 0
        call get_environment_variable('RANK', v, status=st)
        if (st == 0) read(v, *) r
        call get_environment_variable('WORLD_SIZE', v, status=st)
        if (st == 0) read(v, *) n
        call get_environment_variable('LOCAL_RANK', v, status=st)
        if (st == 0) read(v, *) dev
#endif
        if (r < 0 .or. r >= n) then
            write(*, '(a,i0,a,i0)') 'ocn_sw_driver: bad rank ', r, ' of ', n
            error stop 2
        endif
    end subroutine

    subroutine ranks_finalize()
#ifdef OCN_MPI
        call mpi_finalize(ierr)
#endif
    end subroutine

    ! rank 0 makes the RCCL unique id; every rank ends up holding it (mpi_bcast, or a file rank 0
    ! writes under a temporary name and renames -- the others wait for the name to appear)
    subroutine share_unique_id()
        character(len=512) :: path, port
        integer :: st, uu, tries
        logical :: there
        if (rank == 0) call ocn_check(ocn_comm_unique_id(c_loc(uid), int(OCN_UNIQUE_ID_BYTES, c_int32_t)), &
                                      'ocn_comm_unique_id')
        if (nranks == 1) return
#ifdef OCN_MPI
        call mpi_bcast(uid, OCN_UNIQUE_ID_BYTES, MPI_BYTE, 0, MPI_COMM_WORLD, ierr)
#else
        call get_environment_variable('OCN_UID_FILE', path, status=st)
        if (st /= 0) then
            call get_environment_variable('MASTER_PORT', port, status=st)
            if (st /= 0) port = '0'
            path = 'ocn_uid_' // trim(port) // '.bin'
        endif
        if (rank == 0) then
            open(newunit=uu, file=trim(path) // '.tmp', access='stream', form='unformatted', status='replace')
            write(uu) uid
            close(uu)
            if (c_rename(trim(path) // '.tmp' // c_null_char, trim(path) // c_null_char) /= 0) then
                write(*, '(a)') 'ocn_sw_driver: cannot publish the RCCL unique id at ' // trim(path)
                error stop 2
            endif
        else
            do tries = 1, 1200   ! 120 s
                inquire(file=trim(path), exist=there)
                if (there) exit
                st = c_usleep(100000_c_int)
            enddo
            if (.not. there) then
                write(*, '(a)') 'ocn_sw_driver: no RCCL unique id from rank 0 at ' // trim(path)
                error stop 2
            endif
            open(newunit=uu, file=trim(path), access='stream', form='unformatted', status='old', action='read')
            read(uu) uid
            close(uu)
        endif
#endif
    end subroutine

    ! host only: this rank's blocks (ocn_decompose) and the copies / messages of one exchange of the
    ! fields the reference's first sync point sends plus the state (ocn_halo_schedule), as text
    subroutine write_plan(fname)
        character(*), intent(in) :: fname
        type(ocn_block_info), allocatable, target :: blk(:)
        type(ocn_halo_msg), allocatable, target :: msg(:)
        integer(c_int32_t), target :: ids(4) = [OCN_SSHN, OCN_SSH, OCN_UBRTR, OCN_VBRTR]
        integer(c_int32_t) :: n
        type(c_ptr) :: mp
        integer :: uu, i
        mp = c_null_ptr
        if (allocated(mask)) mp = c_loc(mask)
        call ocn_check(ocn_decompose(basin, dec, mp, c_null_ptr, 0_c_int32_t, n), 'ocn_decompose')
        allocate(blk(max(1, n)))
        call ocn_check(ocn_decompose(basin, dec, mp, c_loc(blk), n, n), 'ocn_decompose')
        open(newunit=uu, file=fname, status='replace', action='write')
        write(uu, '(a,i0,a,i0,a,i0)') 'rank ', rank, ' of ', nranks, ' blocks ', n
        do i = 1, n
            write(uu, '(a,22(1x,i0))') 'block', blk(i)%bm, blk(i)%bn, blk(i)%geom%nx_start, blk(i)%geom%nx_end, &
                blk(i)%geom%ny_start, blk(i)%geom%ny_end, blk(i)%nbr_rank, blk(i)%nbr_k
        enddo
        call ocn_check(ocn_halo_schedule(basin, dec, mp, c_loc(ids), 4_c_int32_t, c_null_ptr, 0_c_int32_t, n), &
                       'ocn_halo_schedule')
        allocate(msg(max(1, n)))
        call ocn_check(ocn_halo_schedule(basin, dec, mp, c_loc(ids), 4_c_int32_t, c_loc(msg), n, n), &
                       'ocn_halo_schedule')
        write(uu, '(a,i0)') 'messages ', n
        do i = 1, n
            write(uu, '(a,14(1x,i0),1x,i0)') 'msg', msg(i)%kind, msg(i)%peer, msg(i)%k, msg(i)%k_src, msg(i)%field, &
                msg(i)%dst_x0, msg(i)%dst_x1, msg(i)%dst_y0, msg(i)%dst_y1, msg(i)%src_x0, msg(i)%src_x1, &
                msg(i)%src_y0, msg(i)%src_y1, msg(i)%count, msg(i)%offset
        enddo
        close(uu)
    end subroutine

    ! legacy/service/read_write_parameters.f90:7-42 semantics: first lexeme of each line
    subroutine read_par(fname, out, n)
        character(*), intent(in) :: fname
        character(len=256), intent(out) :: out(:)
        integer, intent(out) :: n
        character(len=512) :: ln
        integer :: uu, ios, p
        out = ''
        n = 0
        open(newunit=uu, file=fname, status='old', action='read')
        do
            read(uu, '(a)', iostat=ios) ln
            if (ios /= 0) exit
            n = n + 1
            if (n > size(out)) exit
            ln = adjustl(ln)
            p = scan(ln, ' :')
            if (p > 1) then
                out(n) = ln(1:p - 1)
            else
                out(n) = trim(ln)
            endif
        enddo
        close(uu)
    end subroutine

    ! tools/io.f90:61-70: a comment line, then ny rows of nx digits, top row (n = ny) first
    subroutine read_mask(fname, nx, ny, m)
        character(*), intent(in) :: fname
        integer, intent(in) :: nx, ny
        integer(c_int32_t), intent(out) :: m(nx, ny)
        character(len=16) :: frmt
        character(len=80) :: comment
        integer :: uu, i, j
        write(frmt, '(a,i9,a)') '(', nx, 'i1)'
        open(newunit=uu, file=fname, status='old', action='read')
        read(uu, '(a)') comment
        do j = ny, 1, -1
            read(uu, frmt) (m(i, j), i = 1, nx)
        enddo
        close(uu)
    end subroutine

end program ocn_sw_driver
