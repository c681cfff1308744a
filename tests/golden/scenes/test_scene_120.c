#include <stdio.h>
#include <string.h>
#include <stdbool.h>
#include <math.h>
#include <unistd.h>

#include "src/libs/canvas/canvas.h"
#include "src/libs/linalg/linalg.h"
#include "src/libs/obj_loader/obj_loader.h"
#include "src/libs/photon_map/pm.h"
#include "src/color/hsl.h"
#include "src/color/lab.h"
#include "src/color/rgb.h"
#include "src/color/srgb.h"
#include "src/color/xyz.h"
#include "src/color/xyy.h"

#include "src/renderer/camera.h"
#include "src/renderer/config.h"
#include "src/renderer/photon_tracer.h"
#include "src/renderer/renderer.h"
#include "src/renderer/world.h"
#include "src/pattern/pattern.h"
#include "src/shapes/shapes.h"
#include "src/shapes/cone.h"
#include "src/shapes/csg.h"
#include "src/shapes/cube.h"
#include "src/shapes/cylinder.h"
#include "src/shapes/group.h"
#include "src/shapes/plane.h"
#include "src/shapes/sphere.h"
#include "src/shapes/triangle.h"
#include "src/shapes/toroid.h"

#define True true
#define False false

int
main()
{
    /* config */
    struct global_config global_config;
    global_config.illumination.include_direct = True;
    global_config.illumination.include_global = False;
    global_config.illumination.debug_visualize_photon_map = False;
    global_config.illumination.debug_visualize_soft_indirect = False;
    global_config.illumination.di.include_ambient = True;
    global_config.illumination.di.include_diffuse = True;
    global_config.illumination.di.include_specular_highlight = True;
    global_config.illumination.di.include_specular = True;
    global_config.illumination.di.path_length = 5;

    global_config.illumination.gi.include_caustics = False;
    global_config.illumination.gi.include_final_gather = False;
    global_config.illumination.gi.usteps = 1;
    global_config.illumination.gi.vsteps = 1;
    global_config.illumination.gi.irradiance_estimate_num = 200;
    global_config.illumination.gi.irradiance_estimate_radius = 0.1000000000;
    global_config.illumination.gi.irradiance_estimate_cone_filter_k = 1.0000000000;
    global_config.illumination.gi.photon_count = 0;
    global_config.illumination.gi.path_length = 5;

    global_config.threading.num_threads = 8;
    global_config.scene.divide_threshold = 1;
    global_config.output.file_path = "/tmp/frt_golden/out/test_scene_120";
    global_config.output.color_space = SRGB;

    void (*color_space_fn)(const Color, Color) = NULL;
    switch (global_config.output.color_space) {
    case RGB:
        color_space_fn = rgb_to_rgb;
        break;
    case HSL:
        color_space_fn = hsl_to_rgb;
        break;
    case XYZ:
        color_space_fn = xyz_to_rgb;
        break;
    case XYY:
        color_space_fn = xyy_to_rgb;
        break;
    case LAB:
        color_space_fn = lab_to_rgb;
        break;
    case SRGB:
        // this is the default
    default:
        color_space_fn = srgb_to_rgb;
        break;
    }

    /* end config */

    /* camera */
    struct aperture ap;
    aperture(POINT_APERTURE, 0.0, 1, 1, false, &ap);

    Point from = { -2.0000000000, 3.0000000000, -6.0000000000, 1.0 };
    Point to = { 0.0000000000, 0.0000000000, 0.0000000000, 1.0 };
    Vector up = { 0.0000000000, 1.0000000000, 0.0000000000, 0.0 };
    Matrix camera_xform;
    view_transform(from, to, up, camera_xform);

    Camera cam = camera(120, 120, 0.5000000000/*field_of_view*/, 1.0000000000/*distance*/, 1/*usteps*/, 1/*vsteps*/, &ap, camera_xform);

    /* end camera */

    /* lights */
    Light all_lights = array_of_lights(1);

    /* point light 0 */
    Light point_light_0 = all_lights + 0;
    Point point_light_0_point = { 2.0000000000, 10.0000000000, -2.0000000000, 1.0 };
    Color point_light_0_intensity = color(1.0000000000, 1.0000000000, 1.0000000000);
    point_light(point_light_0_point, point_light_0_intensity, point_light_0);

    /* end point light 0 */

    /* end lights */

    /* shapes */
    Shape all_shapes = array_of_shapes(2);

    /* shape 0 */
    
        Pattern pattern_0_Ka = NULL;
    Pattern pattern_0_Kd = NULL;
    Pattern pattern_0_Ks = NULL;
    Pattern pattern_0_Ns = NULL;
    Pattern pattern_0_bump = NULL;
    Pattern pattern_0_disp = NULL;
    Pattern pattern_0_refl = NULL;
    Pattern pattern_0_d = NULL;
    Color material_0_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_0_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_0_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_0 = material_alloc();
    color_space_fn(material_0_color_raw, material_0->Ka);
    color_space_fn(material_0_color_raw, material_0->Kd);
    color_space_fn(material_0_color_raw, material_0->Ks);
    color_scale(material_0->Ka, 1.0000000000);
    color_scale(material_0->Kd, 0.0000000000);
    color_scale(material_0->Ks, 0.0000000000);
    rgb_to_rgb(material_0_reflective, material_0->refl);
    rgb_to_rgb(material_0_refractive, material_0->Tf);
    material_0->reflective = material_0_reflective[0] > 0.0
                             || material_0_reflective[1] > 0.0
                             || material_0_reflective[2] > 0.0;

    material_0->Tr = 0.0000000000;
    material_0->Ns = 200.0000000000;
    material_0->Ni = 1.0000000000;
    material_0->casts_shadow = true;
    material_set_pattern(material_0, map_Ka, pattern_0_Ka);
    material_set_pattern(material_0, map_Kd, pattern_0_Kd);
    material_set_pattern(material_0, map_Ks, pattern_0_Ks);
    material_set_pattern(material_0, map_Ns, pattern_0_Ns);
    material_set_pattern(material_0, map_d, pattern_0_d);
    material_set_pattern(material_0, map_bump, pattern_0_bump);
    material_set_pattern(material_0, map_disp, pattern_0_disp);
    material_set_pattern(material_0, map_refl, pattern_0_refl);

    Matrix transform_0, transform_0_tmp;
    matrix_identity(transform_0);
    matrix_rotate_x(1.5708000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);
    matrix_translate(0.0000000000, 0.0000000000, 100.0000000000, transform_0_tmp);
    transform_chain(transform_0_tmp, transform_0);

    Shape shape_0 = all_shapes + 0;
    plane(shape_0);
    shape_set_material(shape_0, material_0);
    shape_set_transform(shape_0, transform_0);

    /* end shape 0 */
    /* shape 1 */
    
    /* children for 1 */
    Shape shape_1_children = array_of_shapes(2);
    
        Pattern pattern_1_left_Ka = NULL;
    Pattern pattern_1_left_Kd = NULL;
    Pattern pattern_1_left_Ks = NULL;
    Pattern pattern_1_left_Ns = NULL;
    Pattern pattern_1_left_bump = NULL;
    Pattern pattern_1_left_disp = NULL;
    Pattern pattern_1_left_refl = NULL;
    Pattern pattern_1_left_d = NULL;
    Color material_1_left_color_raw = color(1.0000000000, 1.0000000000, 0.0000000000);
    Color material_1_left_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_left_refractive = color(0.0000000000, 0.0000000000, 0.0000000000);

    Material material_1_left = material_alloc();
    color_space_fn(material_1_left_color_raw, material_1_left->Ka);
    color_space_fn(material_1_left_color_raw, material_1_left->Kd);
    color_space_fn(material_1_left_color_raw, material_1_left->Ks);
    color_scale(material_1_left->Ka, 0.1000000000);
    color_scale(material_1_left->Kd, 0.9000000000);
    color_scale(material_1_left->Ks, 0.9000000000);
    rgb_to_rgb(material_1_left_reflective, material_1_left->refl);
    rgb_to_rgb(material_1_left_refractive, material_1_left->Tf);
    material_1_left->reflective = material_1_left_reflective[0] > 0.0
                             || material_1_left_reflective[1] > 0.0
                             || material_1_left_reflective[2] > 0.0;

    material_1_left->Tr = 0.0000000000;
    material_1_left->Ns = 200.0000000000;
    material_1_left->Ni = 1.0000000000;
    material_1_left->casts_shadow = true;
    material_set_pattern(material_1_left, map_Ka, pattern_1_left_Ka);
    material_set_pattern(material_1_left, map_Kd, pattern_1_left_Kd);
    material_set_pattern(material_1_left, map_Ks, pattern_1_left_Ks);
    material_set_pattern(material_1_left, map_Ns, pattern_1_left_Ns);
    material_set_pattern(material_1_left, map_d, pattern_1_left_d);
    material_set_pattern(material_1_left, map_bump, pattern_1_left_bump);
    material_set_pattern(material_1_left, map_disp, pattern_1_left_disp);
    material_set_pattern(material_1_left, map_refl, pattern_1_left_refl);

    Matrix transform_1_left;
    matrix_identity(transform_1_left);
    Shape shape_1_left = shape_1_children + 0;
    cube(shape_1_left);
    shape_set_material(shape_1_left, material_1_left);
    shape_set_transform(shape_1_left, transform_1_left);
    
        Pattern pattern_1_right_Ka = NULL;
    Pattern pattern_1_right_Kd = NULL;
    Pattern pattern_1_right_Ks = NULL;
    Pattern pattern_1_right_Ns = NULL;
    Pattern pattern_1_right_bump = NULL;
    Pattern pattern_1_right_disp = NULL;
    Pattern pattern_1_right_refl = NULL;
    Pattern pattern_1_right_d = NULL;
    Color material_1_right_color_raw = color(1.0000000000, 1.0000000000, 1.0000000000);
    Color material_1_right_reflective = color(0.0000000000, 0.0000000000, 0.0000000000);
    Color material_1_right_refractive = color(1.0000000000, 1.0000000000, 1.0000000000);

    Material material_1_right = material_alloc();
    color_space_fn(material_1_right_color_raw, material_1_right->Ka);
    color_space_fn(material_1_right_color_raw, material_1_right->Kd);
    color_space_fn(material_1_right_color_raw, material_1_right->Ks);
    color_scale(material_1_right->Ka, 0.0000000000);
    color_scale(material_1_right->Kd, 0.0000000000);
    color_scale(material_1_right->Ks, 0.0000000000);
    rgb_to_rgb(material_1_right_reflective, material_1_right->refl);
    rgb_to_rgb(material_1_right_refractive, material_1_right->Tf);
    material_1_right->reflective = material_1_right_reflective[0] > 0.0
                             || material_1_right_reflective[1] > 0.0
                             || material_1_right_reflective[2] > 0.0;

    material_1_right->Tr = 1.0000000000;
    material_1_right->Ns = 200.0000000000;
    material_1_right->Ni = 1.0000000000;
    material_1_right->casts_shadow = true;
    material_set_pattern(material_1_right, map_Ka, pattern_1_right_Ka);
    material_set_pattern(material_1_right, map_Kd, pattern_1_right_Kd);
    material_set_pattern(material_1_right, map_Ks, pattern_1_right_Ks);
    material_set_pattern(material_1_right, map_Ns, pattern_1_right_Ns);
    material_set_pattern(material_1_right, map_d, pattern_1_right_d);
    material_set_pattern(material_1_right, map_bump, pattern_1_right_bump);
    material_set_pattern(material_1_right, map_disp, pattern_1_right_disp);
    material_set_pattern(material_1_right, map_refl, pattern_1_right_refl);

    Matrix transform_1_right;
    matrix_translate(0.2000000000, 0.5000000000, -0.3000000000, transform_1_right);
    Shape shape_1_right = shape_1_children + 1;
    sphere(shape_1_right);
    shape_set_material(shape_1_right, material_1_right);
    shape_set_transform(shape_1_right, transform_1_right);

    /* end children for 1 */

    Matrix transform_1;
    matrix_identity(transform_1);
    Shape shape_1 = all_shapes + 1;
    csg(shape_1, CSG_DIFFERENCE, shape_1_left, shape_1_right);
    shape_set_transform(shape_1, transform_1);

    /* end shape 1 */
    /* end shapes */

    Shape world_group = array_of_shapes(1);
    group(world_group, all_shapes, 2);
    printf("Balancing scene...");
    fflush(stdout);
    world_group->divide(world_group, global_config.scene.divide_threshold);
    printf("Done!\n");
    fflush(stdout);

    World w = world();
    w->lights = all_lights;
    w->lights_num = 1;
    w->shapes = world_group;
    w->shapes_num = 1;
    w->global_config = &global_config;

    if (global_config.illumination.gi.photon_count > 0 && (global_config.illumination.include_global  || global_config.illumination.debug_visualize_photon_map || global_config.illumination.debug_visualize_soft_indirect)) {
        w->photon_maps = array_of_photon_maps(3);
        printf("Tracing photons...");
        fflush(stdout);
        int i;
        for (i = 0; i < 3; ++i) {
            init_Photon_map(global_config.illumination.gi.photon_count, w->photon_maps + i);
        }
        trace_photons(w, 3, global_config.illumination.gi.include_caustics, global_config.illumination.gi.include_final_gather);
        printf("Done!\n");
        fflush(stdout);
    } else {
        w->photon_maps = NULL;
        printf("Skipping photon tracing because photon_count is 0.\n");
        fflush(stdout);
    }

    Canvas c = render_multi(cam, w, cam->usteps, cam->vsteps, cam->aperture.jitter);

    write_ppm_file(c, true, global_config.output.file_path);
    write_png(c, global_config.output.file_path);

    canvas_free(c);

    return 0;
}

